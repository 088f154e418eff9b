#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py tests/test_models_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/conv_tests.log 2>&1; rc=$?
tail -5 gpurun_out/conv_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_r50.log 2>&1; rc=$?
grep -E "warmup step 1/|metric" gpurun_out/bench_r50.log; [ $rc -eq 0 ] || exit $rc
PDT_CONV1X1=miopen timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_r50_miopen.log 2>&1; rc=$?
grep -E "metric" gpurun_out/bench_r50_miopen.log; exit $rc
