#!/bin/bash
# ResNet-50 per-GPU batch beyond 512 (288 GB HBM): search conv algorithms (MIOpen find-db) and
# GEMM solutions (TunableOp) for the new shapes, then time read-only runs. Harvests both caches
# into gpurun_out/ for committing.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
rm -rf gpurun_out/miopen_cache; cp -r miopen_cache gpurun_out/miopen_cache
export PDT_MIOPEN_CACHE=$PWD/gpurun_out/miopen_cache
(while sleep 50; do date +%T >> gpurun_out/bb_heartbeat.log; done) & HB=$!
trap 'kill $HB' EXIT
run() { n=$1; t=$2; shift 2; timeout -k 10 $t python -u bench.py "$@" > gpurun_out/bb_$n.log 2>&1; rc=$?
  echo "$n rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/bb_$n.log) $(grep -o 'warmup step 1/[0-9]* done at [0-9.]*' gpurun_out/bb_$n.log)"
  [ $rc -ne 0 ] && tail -5 gpurun_out/bb_$n.log; return $rc; }
for b in ${BATCHES:-1024 768}; do
  rm -rf gpurun_out/tune_b$b; mkdir -p gpurun_out/tune_b$b
  PDT_TUNE_GEMMS=1 PDT_TUNE_GEMMS_OUT=$PWD/gpurun_out/tune_b$b run tune$b ${TUNE_T:-600} --batch-size $b --steps 3 --warmup 2 || exit 1
  cp gpurun_out/tune_b$b/tunableop0.csv tuning/tunableop_gfx950.csv
  run ro$b 200 --batch-size $b --steps 15 --warmup 5 || exit 1
done
run ro512 170 --batch-size 512 --steps 15 --warmup 5 || exit 1
