#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out/r6
timeout -k 10 400 python -u -m pytest tests/test_bwd_alg_gpu.py tests/test_gemm_gpu.py -q --timeout 180 --timeout-method thread > gpurun_out/r6/j_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed|^E  " gpurun_out/r6/j_tests.log | tail -20
[ $rc -le 1 ] || exit $rc
for v in 1 0 1 0; do
PDT_BWD_ALG_FIRST=$v timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6/j_bench_f$v.log 2>&1 || exit 1; echo "bench alg_first=$v $(grep -o '"value": [0-9.]*' gpurun_out/r6/j_bench_f$v.log)"
done
PDT_BWD_ALG_FIRST=1 PC_CFGS="f1:" bash tools/gpu_prof_calls.sh || exit 1
cp gpurun_out/calls_f1.md gpurun_out/steady_f1.md gpurun_out/r6/
