#!/bin/bash
# All GPU tests + the three ours-benches.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/ -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; grep -E "^FAILED|Error" gpurun_out/pytest_gpu.log | head -5
if [ $rc -gt 1 ]; then exit $rc; fi
run() { n=$1; shift; timeout -k 10 500 python bench.py "$@" > gpurun_out/b_$n.log 2>&1; rc=$?
  echo "$n rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/b_$n.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/b_$n.log) $(grep -o '"final_loss": [-0-9.a-zA-Z]*' gpurun_out/b_$n.log)"
  [ $rc -ne 0 ] && tail -5 gpurun_out/b_$n.log; return $rc; }
run rn50_ours --steps 20 --warmup 5 || exit 1
run gpt_ours --model gpt2_medium --steps 10 --warmup 3 || exit 1
run vit_ours --model vit_b16 --steps 10 --warmup 3 || exit 1
