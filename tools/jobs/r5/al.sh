#!/bin/bash
# Round 5 (al): fp8 producers with the transposed (1) / row-major (2) / both (3) stores dropped.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
for pr in 0 1 2 3; do
  echo "== PDT_FP8_STORE_PROBE=$pr"
  PDT_FP8_STORE_PROBE=$pr timeout -k 10 200 python3 tools/fp8_cast_bench.py > gpurun_out/fp8_store_probe_$pr.txt 2>&1 || exit 1
  grep -v amdgpu.ids gpurun_out/fp8_store_probe_$pr.txt | grep -v "^kernel" | head -5
done
