#!/bin/bash
# Stem conv: GPU tests + microbench (run via gpurun from the repo root).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_conv_gpu.py -k stem \
  > gpurun_out/stem_tests.log 2>&1 || { tail -30 gpurun_out/stem_tests.log; exit 1; }
tail -3 gpurun_out/stem_tests.log
PYTHONPATH=. timeout -k 10 240 python -u tools/stem_bench.py 512 2>&1 | tee gpurun_out/stem_bench.log
