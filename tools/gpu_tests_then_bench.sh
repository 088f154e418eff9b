#!/bin/bash
# New/changed GPU tests first (fast feedback), then the whole GPU tier, then the default bench.
# Usage: tools/gpu_tests_then_bench.sh "<pytest node ids of the first tier>"
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
if [ -n "$1" ]; then
  timeout -k 10 900 python -u -m pytest $1 -x -v --timeout 180 --timeout-method thread > gpurun_out/t1_pytest.log 2>&1
  rc=$?; echo "tier1 rc=$rc"; tail -5 gpurun_out/t1_pytest.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 1500 python -u -m pytest tests/ -q -m gpu --timeout 180 --timeout-method thread > gpurun_out/t2_pytest.log 2>&1
rc=$?; echo "full rc=$rc"; tail -8 gpurun_out/t2_pytest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_default.log 2>&1
brc=$?; echo "bench rc=$brc"; grep -E "metric|warmup step 1/" gpurun_out/bench_default.log; exit $brc
