#!/bin/bash
# Stem kernels end to end: GPU tests (conv + profile gate) then the 1-GPU bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_conv_gpu.py -k stem \
  tests/test_profile_gate_gpu.py > gpurun_out/stem_full_tests.log 2>&1 || { tail -30 gpurun_out/stem_full_tests.log; exit 1; }
tail -3 gpurun_out/stem_full_tests.log
timeout -k 10 400 python bench.py > gpurun_out/bench_stem.log 2>&1 || { tail -20 gpurun_out/bench_stem.log; exit 1; }
tail -1 gpurun_out/bench_stem.log
