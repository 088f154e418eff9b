#!/bin/bash
# BN-backward reduction in the dgrad epilogues: kernel/module tests, then in-process A/B on ResNet-50.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv1x1_ours_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/bnbwd_tests.log 2>&1
rc=$?; tail -3 gpurun_out/bnbwd_tests.log; [ $rc -eq 0 ] || { grep -E "Error|error|assert" gpurun_out/bnbwd_tests.log | head -20; exit $rc; }
timeout -k 10 600 python -u tools/ab_env.py --reps 2 --configs 'on:PDT_BN_BWD_STATS=1' 'off:PDT_BN_BWD_STATS=0' --steps 10 --warmup 3 > gpurun_out/ab_bnbwd.log 2>&1
rc=$?; grep "\[ab\]" gpurun_out/ab_bnbwd.log; exit $rc
