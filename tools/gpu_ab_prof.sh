#!/bin/bash
# Steady-state kernel profiles of the default bench under two values of one switch, then the per-kernel diff.
# Usage: tools/gpu_ab_prof.sh VAR "A-value" "B-value" [extra bench args]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
var=$1; a=$2; b=$3; shift 3
for v in "$a" "$b"; do
  rm -rf /tmp/p_ab_$v; mkdir -p /tmp/p_ab_$v
  export $var="$v"
  timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --output-format csv -d /tmp/p_ab_$v -o run -- python3 bench.py --steps 5 --warmup 3 "$@" > gpurun_out/abprof_${var}_$v.log 2>&1
  rc=$?; echo "$var=$v prof rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/abprof_${var}_$v.log)"; [ $rc -eq 0 ] || exit $rc
  python tools/prof_window.py /tmp/p_ab_$v gpurun_out/abprof_${var}_$v timed 5 > /dev/null || exit 1
done
python tools/prof_diff.py gpurun_out/abprof_${var}_${a}_kernels.csv gpurun_out/abprof_${var}_${b}_kernels.csv 5 30 > gpurun_out/abprof_${var}_diff.md
head -34 gpurun_out/abprof_${var}_diff.md
