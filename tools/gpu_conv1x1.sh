#!/bin/bash
# Our 1x1-conv GEMM: numerics tests, per-shape microbenchmark, then the ResNet-50 bench with it
# on (default) and off.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_conv1x1_ours_gpu.py tests/test_conv_gpu.py > gpurun_out/c1_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/c1_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/conv1x1_bench.py > gpurun_out/c1_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; cat gpurun_out/c1_bench.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/c1_r50_on.log 2>&1
rc=$?; echo "r50 on rc=$rc"; grep -o '"value": [0-9.]*' gpurun_out/c1_r50_on.log; [ $rc -eq 0 ] || exit $rc
PDT_CONV1X1_OURS=none timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/c1_r50_off.log 2>&1
rc=$?; echo "r50 off rc=$rc"; grep -o '"value": [0-9.]*' gpurun_out/c1_r50_off.log; exit $rc
