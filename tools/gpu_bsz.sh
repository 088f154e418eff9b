#!/bin/bash
# ResNet-50 per-GPU batch sweep on the current tree (fresh process per size, driver-style bench).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
for b in ${SIZES:-768 1024}; do
  timeout -k 10 500 python -u bench.py --batch-size $b --steps 20 --warmup 5 > gpurun_out/bench_b$b.log 2>&1
  rc=$?; echo "batch $b rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/bench_b$b.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_b$b.log) first-step: $(grep -o 'warmup step 1/5 done at [0-9.]*s' gpurun_out/bench_b$b.log)"
  [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_b$b.log; exit $rc; }
done
