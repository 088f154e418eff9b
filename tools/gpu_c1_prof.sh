#!/bin/bash
# 1x1/3x3 statistics-epilogue tests, then the ResNet-50 bench + steady-state kernel profile.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_conv1x1_ours_gpu.py > gpurun_out/c1_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/c1_tests.log; [ $rc -eq 0 ] || exit $rc
TAG=${TAG:-_c1} bash tools/gpu_prof_r50.sh
