#!/bin/bash
# Extend the GEMM tuning table with the gradient-accumulation ViT shapes and LeNet.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
run() { n=$1; shift; timeout -k 10 600 python -u bench.py "$@" > gpurun_out/tg_$n.log 2>&1; rc=$?
  echo "$n rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/tg_$n.log) $(grep -o 'warmup step 1/[0-9]* done at [0-9.]*' gpurun_out/tg_$n.log)"
  [ $rc -ne 0 ] && tail -5 gpurun_out/tg_$n.log; return $rc; }
for spec in "vitacc:--model vit_b16 --grad-accum 4" "vitacc8:--model vit_b16 --grad-accum 4 --precision fp8" "lenet:--model lenet"; do
  n=${spec%%:*}; extra=${spec#*:}
  rm -rf gpurun_out/tune_$n; mkdir -p gpurun_out/tune_$n
  PDT_TUNE_GEMMS=1 PDT_TUNE_GEMMS_OUT=$PWD/gpurun_out/tune_$n run ${n}_tune --steps 5 --warmup 2 $extra || exit 1
  run ${n}_tuned --steps 10 --warmup 3 $extra || exit 1
done
