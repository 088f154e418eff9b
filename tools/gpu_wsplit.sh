#!/bin/bash
# Split-K 1x1 weight gradients: tests, then in-process A/B against MIOpen/hipBLASLt table choices.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv1x1_ours_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/wsplit_tests.log 2>&1
rc=$?; tail -2 gpurun_out/wsplit_tests.log; [ $rc -eq 0 ] || { grep -E "Error|error|assert|FAILED" gpurun_out/wsplit_tests.log | head -20; exit $rc; }
timeout -k 10 700 python -u tools/ab_env.py --reps 3 --configs 'splitk:' 'lib:PDT_WGRAD_SPLITK=0' --steps 10 --warmup 3 > gpurun_out/ab_wsplit.log 2>&1
rc=$?; grep "\[ab\]" gpurun_out/ab_wsplit.log; exit $rc
