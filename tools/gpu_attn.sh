#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -k "attention" > gpurun_out/pytest_attn.log 2>&1
rc=$?; echo "attn tests rc=$rc"; grep -E "passed|failed|Error|assert|FAIL|Mismatch|Greatest" gpurun_out/pytest_attn.log | head -20
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 600 python -m pytest tests/ -m gpu -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "all gpu tests rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
run() { n=$1; shift; timeout -k 10 500 python bench.py "$@" > gpurun_out/b_$n.log 2>&1; rc=$?
  echo "$n rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/b_$n.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/b_$n.log) $(grep -o '"final_loss": [-0-9.a-zA-Z]*' gpurun_out/b_$n.log)"
  [ $rc -ne 0 ] && tail -5 gpurun_out/b_$n.log; return $rc; }
run gpt_ours --model gpt2_medium --steps 10 --warmup 3 || exit 1
run gpt_torch --model gpt2_medium --steps 10 --warmup 3 --impl torch_ddp || exit 1
run vit_ours --model vit_b16 --steps 10 --warmup 3 || exit 1
run vit_torch --model vit_b16 --steps 10 --warmup 3 --impl torch_ddp || exit 1
