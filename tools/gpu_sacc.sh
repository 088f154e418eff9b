#!/bin/bash
# Strided shortcut gradient accumulated in conv1's dgrad epilogue: tests, then in-process A/B.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_conv1x1_ours_gpu.py tests/test_conv_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sacc_tests.log 2>&1
rc=$?; tail -2 gpurun_out/sacc_tests.log; [ $rc -eq 0 ] || { grep -E "Error|error|assert|FAILED" gpurun_out/sacc_tests.log | head -20; exit $rc; }
timeout -k 10 700 python -u tools/ab_env.py --reps 2 --configs 'sacc:' 'add:PDT_STRIDED_ACC=0' --steps 10 --warmup 3 > gpurun_out/ab_sacc.log 2>&1
rc=$?; grep "\[ab\]" gpurun_out/ab_sacc.log; exit $rc
