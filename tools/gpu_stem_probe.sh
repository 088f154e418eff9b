#!/bin/bash
# Stem conv probes (tools/convbench/stem_bench.cpp built with PDT_STEM_PROBE=0..3).
set -o pipefail
mkdir -p gpurun_out
for p in 0 1 3; do
  timeout -k 10 60 tools/convbench/stem_bench_p$p 512 2>&1 | tee -a gpurun_out/stem_probe.log || exit 1
done
