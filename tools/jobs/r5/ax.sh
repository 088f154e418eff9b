#!/bin/bash
# Round 5 (ax): LayerNorm backward workgroup cap sweep (PDT_LN_BWD_BLOCKS), per call.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
for c in 512 1024 2048 256 512; do
  PDT_LN_BWD_BLOCKS=$c timeout -k 10 120 python -u tools/ln_bwd_bench.py >> gpurun_out/ln_bwd_ax.txt 2>&1; rc=$?
  [ $rc -eq 0 ] || { tail -5 gpurun_out/ln_bwd_ax.txt; exit $rc; }
done
grep '^{' gpurun_out/ln_bwd_ax.txt
