#!/bin/bash
# Default bench (driver command shape) under two values of one switch, same box, back to back.
# Usage: tools/gpu_ab_bench.sh VAR "on-value" "off-value" [extra bench args]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
var=$1; on=$2; off=$3; shift 3
for v in "$on" "$off" "$on"; do
  env $var="$v" timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 "$@" > gpurun_out/ab_${var}_${v}.log 2>&1
  rc=$?; echo "$var=$v rc=$rc: $(grep -o '"value": [0-9.]*' gpurun_out/ab_${var}_${v}.log) $(grep -o '"comm_exposed_ms": [0-9.a-z]*' gpurun_out/ab_${var}_${v}.log)"
  [ $rc -eq 0 ] || exit $rc
done
