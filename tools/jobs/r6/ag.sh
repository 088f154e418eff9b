#!/bin/bash
# z3 never written + bn3 apply as the APPLY GEMM on layers 1 / 1-2 (PDT_Z3_VIRTUAL=2 with PDT_BN_APPLY_GEMM_K 64 / 128)
# against the default (K = 0: plain apply pass, z3 written)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out/r6
for cfg in 0:0 2:64 2:128 0:0 2:64 2:128; do
  v=${cfg%%:*}; k=${cfg##*:}
  PDT_Z3_VIRTUAL=$v PDT_BN_APPLY_GEMM_K=$k timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r6/ag_${v}_$k.log 2>&1 || exit 3
  echo "z3_virtual=$v apply_gemm_k=$k $(grep -o '"value": [0-9.]*' gpurun_out/r6/ag_${v}_$k.log)"
done
