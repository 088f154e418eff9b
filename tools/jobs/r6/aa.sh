#!/bin/bash
# with G's hi half only: PDT_DS_ALG 512 vs 2048 (b1024), PDT_BWD_ALG_MIN_M 50176 vs 25088 (b128 graphed)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out/r6
for v in 512 2048 512 2048; do
  PDT_DS_ALG=$v timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r6/aa_bench_$v.log 2>&1 || exit 3
  echo "ds_alg=$v b1024 $(grep -o '"value": [0-9.]*' gpurun_out/r6/aa_bench_$v.log)"
done
for m in 50176 25088 50176 25088; do
  PDT_BWD_ALG_MIN_M=$m timeout -k 10 300 python3 bench.py --global-batch 128 --steps 30 --warmup 5 --graph 1 > gpurun_out/r6/aa_b128_$m.log 2>&1 || exit 3
  echo "min_m=$m b128 graph $(grep -o '"value": [0-9.]*' gpurun_out/r6/aa_b128_$m.log)"
done
