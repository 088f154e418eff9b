#!/bin/bash
# Transformer path: LN/attention kernel tests, model numerics, GPT-2 + ViT benches.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_fp8_gpu.py -q -x --timeout 120 --timeout-method thread -k "layernorm or attention or gpt or vit or fp8" > gpurun_out/tx_tests.log 2>&1; rc=$?
tail -3 gpurun_out/tx_tests.log; [ $rc -eq 0 ] || exit $rc
run() { n=$1; shift; timeout -k 10 400 python -u bench.py "$@" > gpurun_out/b_$n.log 2>&1; rc=$?
  echo "$n rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/b_$n.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/b_$n.log)"
  [ $rc -ne 0 ] && tail -5 gpurun_out/b_$n.log; return $rc; }
run gpt_ours --model gpt2_medium --steps 10 --warmup 3 || exit 1
run vit_ours --model vit_b16 --steps 10 --warmup 3 || exit 1
run vit_fp8 --model vit_b16 --steps 10 --warmup 3 --precision fp8 || exit 1
