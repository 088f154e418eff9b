#!/bin/bash
# Stem pool+BN backward fusion and downsample (dy, mask) hand-off: tests, then in-process A/B.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv1x1_ours_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/bnbwd2_tests.log 2>&1
rc=$?; tail -3 gpurun_out/bnbwd2_tests.log; [ $rc -eq 0 ] || { grep -E "Error|error|assert|FAILED" gpurun_out/bnbwd2_tests.log | head -20; exit $rc; }
timeout -k 10 700 python -u tools/ab_env.py --reps 2 --configs 'new:' 'nostem:PDT_STEM_BWD_FUSED=0' 'nods:PDT_DS_MASKED=0' --steps 10 --warmup 3 > gpurun_out/ab_bnbwd2.log 2>&1
rc=$?; grep "\[ab\]" gpurun_out/ab_bnbwd2.log; exit $rc
