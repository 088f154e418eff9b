#!/bin/bash
# Round 5 (as): gemm.hip forced tile widths (PDT_GEMM_BN) on every harness shape.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for bn in 256 128; do
  PDT_GEMM_BN=$bn timeout -k 10 120 tools/convbench/gemmb_p0 > gpurun_out/gemm_as_$bn.txt 2>&1; rc=$?
  echo "== BN=$bn"; grep -v amdgpu.ids gpurun_out/gemm_as_$bn.txt; [ $rc -eq 0 ] || exit $rc
done
