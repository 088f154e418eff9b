#!/bin/bash
# Steady-state ResNet-50 kernel profiles, default and with the env switches in $ALT (A/B by kernel).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
for tag in def alt; do
  rm -rf /tmp/p_$tag; mkdir -p /tmp/p_$tag
  if [ $tag = alt ]; then export $ALT; fi
  timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --output-format csv -d /tmp/p_$tag -o run -- python3 bench.py --steps 5 --warmup 3 > gpurun_out/prof_$tag.log 2>&1
  rc=$?; echo "prof $tag rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/prof_$tag.log)"; [ $rc -eq 0 ] || exit $rc
  python tools/prof_window.py /tmp/p_$tag gpurun_out/steady_$tag timed 5 > /dev/null
  head -1 gpurun_out/steady_$tag.md
done
python tools/prof_diff.py gpurun_out/steady_def_kernels.csv gpurun_out/steady_alt_kernels.csv 5 60 > gpurun_out/prof_diff.md 2>&1; head -30 gpurun_out/prof_diff.md
