#!/bin/bash
# small_gemm 64-row steps: tests + microbench; then the APPLY-GEMM A/B (p.sh)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u -m pytest tests/test_bwd_alg_gpu.py -k "small_gemm or assemble or materialised or determin" -v --timeout 240 --timeout-method thread > gpurun_out/r6/q_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r6/q_tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/alg_bench.py > gpurun_out/r6/q_algbench.log 2>&1 || exit 4
cat gpurun_out/r6/q_algbench.log | grep -v amdgpu.ids
bash tools/jobs/r6/p.sh
