#!/bin/bash
# Round 5 (bd): steady-state windows of GPT-2-medium fp8 and bf16 on the final tree (GPT-2 fp8 GEMMs now in the
# TunableOp table), graphed-step kernels included.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in "gpt2_medium --precision fp8" "gpt2_medium"; do
  tag=$(echo $cfg | tr ' -' '__')
  rm -rf /tmp/p_$tag; mkdir -p /tmp/p_$tag
  timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --output-format csv -d /tmp/p_$tag -o run -- python3 bench.py --model $cfg --steps 5 --warmup 3 > gpurun_out/bd_$tag.log 2>&1
  rc=$?; echo "$cfg prof rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/bd_$tag.log)"; [ $rc -eq 0 ] || exit $rc
  python tools/prof_window.py /tmp/p_$tag gpurun_out/steady_bd_$tag timed 5 > /dev/null && head -1 gpurun_out/steady_bd_$tag.md || exit 1
  python tools/prof_categories.py gpurun_out/steady_bd_${tag}_kernels.csv > gpurun_out/steady_bd_${tag}_categories.md 2>/dev/null || true
done
