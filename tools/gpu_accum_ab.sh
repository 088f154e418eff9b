#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
run() { n=$1; shift; timeout -k 10 500 python -u bench.py "$@" > gpurun_out/ac_$n.log 2>&1; rc=$?
  echo "$n rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/ac_$n.log)"; [ $rc -ne 0 ] && tail -5 gpurun_out/ac_$n.log; return $rc; }
run tuned --model vit_b16 --grad-accum 4 --steps 10 --warmup 3 || exit 1
PDT_GEMM_TUNING=0 run plain --model vit_b16 --grad-accum 4 --steps 10 --warmup 3 || exit 1
run tuned2 --model vit_b16 --grad-accum 4 --steps 10 --warmup 3 || exit 1
PDT_GEMM_TUNING=0 run plain2 --model vit_b16 --grad-accum 4 --steps 10 --warmup 3 || exit 1
