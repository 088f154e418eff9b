#!/bin/bash
# BN tile finalize: one launch with a ticket (default) vs two launches (PDT_BN_TILES_FUSED=0), b1024 and b128 graphed
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out/r6
for v in 1 0 1 0; do
  PDT_BN_TILES_FUSED=$v timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r6/af_bench_$v.log 2>&1 || exit 3
  echo "tiles_fused=$v b1024 $(grep -o '"value": [0-9.]*' gpurun_out/r6/af_bench_$v.log)"
done
for v in 1 0; do
  PDT_BN_TILES_FUSED=$v timeout -k 10 300 python3 bench.py --global-batch 128 --steps 30 --warmup 5 --graph 1 > gpurun_out/r6/af_b128_$v.log 2>&1 || exit 3
  echo "tiles_fused=$v b128 graph $(grep -o '"value": [0-9.]*' gpurun_out/r6/af_b128_$v.log)"
done
