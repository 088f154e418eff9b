#!/bin/bash
# Quick check after a model-level change: selected GPU tests then the 1-GPU bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread ${TESTS:-tests/test_models_gpu.py} \
  > gpurun_out/quick_tests.log 2>&1 || { tail -30 gpurun_out/quick_tests.log; exit 1; }
tail -2 gpurun_out/quick_tests.log
timeout -k 10 400 python bench.py > gpurun_out/bench_quick.log 2>&1 || { tail -20 gpurun_out/bench_quick.log; exit 1; }
tail -1 gpurun_out/bench_quick.log | cut -c1-200
