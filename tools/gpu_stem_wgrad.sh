#!/bin/bash
# Stem weight gradient: standalone correctness + timing (tools/convbench/stem_bench.cpp WGRAD=1),
# then the staging-only / compute-only probes when built (stem_bench_w1 / _w2).
set -o pipefail
mkdir -p gpurun_out
WGRAD=1 timeout -k 10 120 tools/convbench/stem_bench_p0 2>&1 | tee gpurun_out/stem_wgrad.log || exit 1
for p in 1 2; do
  [ -x tools/convbench/stem_bench_w$p ] || continue
  echo "probe $p"; WGRAD=1 timeout -k 10 120 tools/convbench/stem_bench_w$p 2>&1 | tail -1 | tee -a gpurun_out/stem_wgrad.log
done
