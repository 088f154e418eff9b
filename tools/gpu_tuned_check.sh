#!/bin/bash
# Read-only tuned-GEMM table (engine/gemm_tuning.py) vs no table, every workload.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
run() { n=$1; shift; timeout -k 10 500 python -u bench.py "$@" > gpurun_out/tc_$n.log 2>&1; rc=$?
  echo "$n rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/tc_$n.log) $(grep -o 'warmup step 1/[0-9]* done at [0-9.]*' gpurun_out/tc_$n.log)"
  [ $rc -ne 0 ] && tail -5 gpurun_out/tc_$n.log; return $rc; }
run r50 --steps 20 --warmup 5 || exit 1
PDT_GEMM_TUNING=0 run r50_plain --steps 20 --warmup 5 || exit 1
run gpt --model gpt2_medium --steps 10 --warmup 3 || exit 1
run vit --model vit_b16 --steps 10 --warmup 3 || exit 1
run vit_fp8 --model vit_b16 --steps 10 --warmup 3 --precision fp8 || exit 1
PDT_GEMM_TUNING=0 run vit_fp8_plain --model vit_b16 --steps 10 --warmup 3 --precision fp8 || exit 1
