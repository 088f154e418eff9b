#!/bin/bash
# Transformer configs: bench (driver command shape) + a rocprofv3 window of the timed steps each.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in ${TX_CFGS:-"gpt2_medium" "gpt2_medium --precision fp8" "vit_b16" "vit_b16 --precision fp8"}; do
  tag=$(echo $cfg | tr ' -' '__')
  timeout -k 10 400 python3 bench.py --model $cfg --gpus 1 --steps 20 --warmup 5 > gpurun_out/tx_$tag.log 2>&1
  rc=$?; echo "$cfg rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/tx_$tag.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/tx_$tag.log)"
  [ $rc -eq 0 ] || exit $rc
  rm -rf /tmp/p_$tag; mkdir -p /tmp/p_$tag
  timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --output-format csv -d /tmp/p_$tag -o run -- python3 bench.py --model $cfg --steps 5 --warmup 3 > gpurun_out/txprof_$tag.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "prof rc=$rc"; exit $rc; }
  python tools/prof_window.py /tmp/p_$tag gpurun_out/steady_$tag timed 5 > /dev/null && head -1 gpurun_out/steady_$tag.md
done
