#!/bin/bash
# Run the given GPU test files (or node ids) in ONE pytest process, then optional extra commands.
# Usage: tools/gpu_tests.sh "<pytest targets>" [log-name]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
log=gpurun_out/${2:-tests}.log
timeout -k 10 900 python -u -m pytest $1 -x -v --timeout 180 --timeout-method thread > $log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" $log | tail -40; exit $rc
