#!/bin/bash
# Iteration run: GPU tests, bench variants for the three north-star models.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/ -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -25 gpurun_out/pytest_gpu.log | grep -E "passed|failed|Error|assert|FAIL" | head
if [ $rc -gt 1 ]; then exit $rc; fi
run() { # name args...
  n=$1; shift
  timeout -k 10 500 python bench.py "$@" > gpurun_out/b_$n.log 2>&1
  rc=$?; echo "$n rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/b_$n.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/b_$n.log) $(grep -o '"final_loss": [-0-9.a-zA-Z]*' gpurun_out/b_$n.log)"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/b_$n.log; fi
  return $rc
}
run rn50_ours --steps 20 --warmup 5 || exit 1
run rn50_torch --steps 20 --warmup 5 --impl torch_ddp || exit 1
run vit_ours --model vit_b16 --steps 10 --warmup 3 || exit 1
run vit_torch --model vit_b16 --steps 10 --warmup 3 --impl torch_ddp || exit 1
run gpt_ours --model gpt2_medium --steps 10 --warmup 3 || exit 1
run gpt_torch --model gpt2_medium --steps 10 --warmup 3 --impl torch_ddp || exit 1
