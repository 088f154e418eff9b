#!/bin/bash
# Stem pool backward: tests, then per-kernel profile default (fused) vs PDT_STEM_BWD_FUSED=0.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_conv1x1_ours_gpu.py -x -q -k "pool or stem" --timeout 120 --timeout-method thread > gpurun_out/stem_tests.log 2>&1
rc=$?; tail -2 gpurun_out/stem_tests.log; [ $rc -eq 0 ] || { grep -E "Error|error|assert|FAILED" gpurun_out/stem_tests.log | head -20; exit $rc; }
ALT=PDT_STEM_BWD_FUSED=0 bash tools/gpu_prof2.sh
