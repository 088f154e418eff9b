#!/bin/bash
# Strided 1x1 shortcut as gather + our GEMM (+BN stats) + split-K weight gradient: tests, then A/B.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s2_tests.log 2>&1
rc=$?; tail -2 gpurun_out/s2_tests.log; [ $rc -eq 0 ] || { grep -E "Error|error|assert|FAILED" gpurun_out/s2_tests.log | head -20; exit $rc; }
timeout -k 10 700 python -u tools/ab_env.py --reps 3 --configs 'miopen_s2:' 'gemm_s2:PDT_CONV1X1_S2=1' --steps 10 --warmup 3 > gpurun_out/ab_s2.log 2>&1
rc=$?; grep "\[ab\]" gpurun_out/ab_s2.log; exit $rc
