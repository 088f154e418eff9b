#!/bin/bash
# Round 5 (az): fp8 vs bf16 with the hipGraph-captured step (host gaps removed), GPT-2-medium and ViT-B/16, same box.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
for m in gpt2_medium vit_b16; do
  for p in bf16 fp8 bf16 fp8; do
    timeout -k 10 400 python -u bench.py --model $m --precision $p --graph 1 --steps 20 --warmup 5 > gpurun_out/az_run.log 2>&1; rc=$?
    echo "$m $p graph rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/az_run.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/az_run.log)" | tee -a gpurun_out/az.txt
    [ $rc -eq 0 ] || { tail -20 gpurun_out/az_run.log; exit $rc; }
  done
done
