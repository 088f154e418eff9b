#!/bin/bash
# Standalone GEMM kernel timings (tools/convbench/gemm_bench.cpp): every prebuilt variant
# tools/convbench/gemm_bench_* (built on the CPU side), one after the other.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for b in tools/convbench/gemm_bench_*; do
  v=$(basename $b)
  timeout -k 10 120 $b > gpurun_out/$v.txt 2>&1
  rc=$?; sed "s/^/$v /" gpurun_out/$v.txt; [ $rc -eq 0 ] || exit $rc
done
