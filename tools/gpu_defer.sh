#!/bin/bash
# Deferred downsample-BN apply: tests, then in-process A/B (ResNet-50, 512/GPU).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_conv1x1_ours_gpu.py tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/defer_tests.log 2>&1
rc=$?; tail -2 gpurun_out/defer_tests.log; [ $rc -eq 0 ] || { grep -E "Error|error|assert|FAILED" gpurun_out/defer_tests.log | head -20; exit $rc; }
timeout -k 10 700 python -u tools/ab_env.py --reps 2 --configs 'defer:' 'write:PDT_DS_DEFER=0' --batch-size 512 --steps 10 --warmup 3 > gpurun_out/ab_defer.log 2>&1
rc=$?; grep "\[ab\]" gpurun_out/ab_defer.log; exit $rc
