#!/bin/bash
# same-box A/B: bn3 apply as the APPLY GEMM in layer 1 (PDT_BN_APPLY_GEMM_K=64, default) vs the standalone apply pass
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out/r6
for k in 64 0 64 0; do
  PDT_BN_APPLY_GEMM_K=$k timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r6/p_bench_$k.log 2>&1 || exit 3
  echo "apply_gemm_k=$k $(grep -o '"value": [0-9.]*' gpurun_out/r6/p_bench_$k.log)"
done
