#!/bin/bash
# Per-call kernel list of one step (tools/prof_calls.py) for the default bench and the 128/GPU graphed step.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in ${PC_CFGS:-b1024: b128:--global-batch,128,--graph,1}; do
  tag=${cfg%%:*}; args=${cfg#*:}; args=${args//,/ }
  rm -rf /tmp/pc_$tag; mkdir -p /tmp/pc_$tag
  timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --output-format csv -d /tmp/pc_$tag -o run -- python3 bench.py --steps 5 --warmup 3 $args > gpurun_out/pc_$tag.log 2>&1
  rc=$?; echo "$tag prof rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/pc_$tag.log)"; [ $rc -eq 0 ] || exit $rc
  python tools/prof_calls.py /tmp/pc_$tag timed 5 > gpurun_out/calls_$tag.md || exit 1
  python tools/prof_window.py /tmp/pc_$tag gpurun_out/steady_$tag timed 5 > /dev/null || exit 1
  tail -1 gpurun_out/calls_$tag.md
done
