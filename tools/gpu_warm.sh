#!/bin/bash
# Driver-style bench (fresh process, committed caches) at the driver's default warm-up and with a longer one.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for w in 5 15; do
  timeout -k 10 400 python -u bench.py --steps 20 --warmup $w > gpurun_out/bench_w$w.log 2>&1
  rc=$?; echo "warmup $w rc=$rc $(grep -o '"value": [0-9.]*, "unit": "images/sec", "n_gpus": 1, "steps": 20, "warmup": [0-9]*, "ms_per_step": [0-9.]*' gpurun_out/bench_w$w.log)"
  grep "warmup step" gpurun_out/bench_w$w.log | tr '\n' ' '; echo
  [ $rc -eq 0 ] || exit $rc
done
