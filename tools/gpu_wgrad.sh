#!/bin/bash
# 3x3 weight-gradient kernel: correctness + timing (new wave map, old map, MFMA-only probe).
set -o pipefail
mkdir -p gpurun_out
WGRAD=1 timeout -k 10 120 tools/convbench/conv3x3_bench 20 2>&1 | tee gpurun_out/wgrad_new.log || exit 1
WGRAD=1 timeout -k 10 120 tools/convbench/conv3x3_bench_c1 20 2>&1 | tee gpurun_out/wgrad_old.log || exit 1
WGRAD=1 PROBE=1 timeout -k 10 120 tools/convbench/conv3x3_bench_p2 20 2>&1 | tee gpurun_out/wgrad_probe2.log
