#!/bin/bash
# End-of-session numbers with the driver's bench command shape, one fresh process per config.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
for cfg in "resnet50" "vit_b16" "gpt2_medium" "vit_b16 --precision fp8"; do
  tag=$(echo $cfg | tr ' -' '__')
  timeout -k 10 500 python3 bench.py --model $cfg --gpus 1 --steps 20 --warmup 5 > gpurun_out/final_$tag.log 2>&1
  rc=$?; echo "$cfg rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/final_$tag.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/final_$tag.log)"
  [ $rc -eq 0 ] || exit $rc
done
