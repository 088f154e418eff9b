#!/bin/bash
# SEG GEMM tile (PDT_SEG_TILE 0 / 1 / 2) with the hi-only G: microbench + bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out/r6
for t in 0 1 2 0 1 2; do
  PDT_SEG_TILE=$t timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r6/ab_bench_$t.log 2>&1 || exit 3
  echo "seg_tile=$t b1024 $(grep -o '"value": [0-9.]*' gpurun_out/r6/ab_bench_$t.log)"
done
