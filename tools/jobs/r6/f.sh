#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out/r6
for cfg in "0 -1" "1 -1" "2 -1" "0 4" "1 4" "0 0" ; do
  set -- $cfg
  PDT_SEG_TILE=$1 PDT_WGRAD_SEG_VARIANT=$2 timeout -k 10 120 python -u tools/alg_bench.py >> gpurun_out/r6/f_alg_bench.log 2>&1 || { echo "fail $cfg"; tail -5 gpurun_out/r6/f_alg_bench.log; exit 1; }
done
grep "\[" gpurun_out/r6/f_alg_bench.log
