#!/bin/bash
# The driver's exact bench command on a fresh box (committed caches only), with a heartbeat file.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_default.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -E "warmup step|metric" gpurun_out/bench_default.log | cut -c1-400; exit $rc
