#!/bin/bash
# Measure the 1x1-conv MIOpen-vs-GEMM decisions for the ResNet-50 bench shapes (512 and 1024 per
# GPU) and dump them as tables (ops/conv.py), timing the bench at the same time.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
rm -rf gpurun_out/miopen_cache; cp -r miopen_cache gpurun_out/miopen_cache
export PDT_MIOPEN_CACHE=$PWD/gpurun_out/miopen_cache
for b in ${BATCHES:-1024 512}; do
  PDT_CONV1X1_TABLE=0 PDT_CONV1X1_DUMP=$PWD/gpurun_out/conv1x1_b$b.json PDT_STACK_DUMP=60 \
    timeout -k 10 ${T:-420} python -u bench.py --batch-size $b --steps 20 --warmup 5 > gpurun_out/ct_b$b.log 2>&1; rc=$?
  echo "b$b rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/ct_b$b.log) $(grep -o 'warmup step 1/[0-9]* done at [0-9.]*' gpurun_out/ct_b$b.log)"
  [ $rc -eq 0 ] || exit $rc
done
