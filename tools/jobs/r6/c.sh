#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out/r6
timeout -k 10 600 python -u -m pytest tests/test_bwd_alg_gpu.py tests/test_conv1x1_ours_gpu.py tests/test_gap_bwd_gpu.py tests/test_conv1x1_persist_gpu.py tests/test_amp_gpu.py "tests/test_gemm_gpu.py::test_linear_per_shape_dispatch" -v --timeout 180 --timeout-method thread > gpurun_out/r6/c_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed|^E  " gpurun_out/r6/c_tests.log | tail -40
[ $rc -le 1 ] || exit $rc
for a in 1 2 0; do
PDT_BWD_ALG=$a timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6/c_bench_alg$a.log 2>&1; echo "bench alg=$a rc=$?"; grep -o '"value": [0-9.]*' gpurun_out/r6/c_bench_alg$a.log
done
timeout -k 10 300 python -u tools/diag_amp16.py > gpurun_out/r6/c_diag_amp16.log 2>&1; echo "diag rc=$?"; grep -v Warning gpurun_out/r6/c_diag_amp16.log | tail -8
