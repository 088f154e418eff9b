#!/bin/bash
# Round 5 (bc): LayerNorm backward minimum rows per workgroup (PDT_LN_BWD_ROWS) at the cap of 512.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/ln_bwd_bc.txt
for r in 32 16 8 32 16; do
  echo "rows=$r" >> gpurun_out/ln_bwd_bc.txt
  PDT_LN_BWD_ROWS=$r timeout -k 10 120 python -u tools/ln_bwd_bench.py >> gpurun_out/ln_bwd_bc.txt 2>&1; rc=$?
  [ $rc -eq 0 ] || { tail -5 gpurun_out/ln_bwd_bc.txt; exit $rc; }
done
grep -v amdgpu.ids gpurun_out/ln_bwd_bc.txt
