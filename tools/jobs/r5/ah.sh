#!/bin/bash
# Round 5 (ah): fp8 producers with / without the per-workgroup amax atomics (cost of the single-word contention).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
for pr in 0 1 0 1; do
  echo "== PDT_FP8_AMAX_PROBE=$pr"
  PDT_FP8_AMAX_PROBE=$pr timeout -k 10 200 python3 tools/fp8_cast_bench.py > gpurun_out/fp8_cast_bench_$pr.txt 2>&1 || exit 1
  grep -v amdgpu.ids gpurun_out/fp8_cast_bench_$pr.txt | grep -v "^kernel"
done
