#!/bin/bash
# graph replay of the 1024/GPU step after allocator churn: which switch makes fc.bias's gradient replay right
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out/r6
run() { tag=$1; shift; env "$@" timeout -k 10 300 python3 -u tools/diag_graph_model.py --batch-size 1024 > gpurun_out/r6/al_$tag.log 2>&1 || { echo "$tag rc=$?"; exit 5; }
  echo "$tag: $(grep -A1 '^replay 1' gpurun_out/r6/al_$tag.log | tail -1)"; }
run minm60000 PDT_BWD_ALG_MIN_M=60000
run global DIAG_CAPMODE=global
run bwdalg0 PDT_BWD_ALG=0
run prep0 PDT_PREP_WEIGHTS=0
