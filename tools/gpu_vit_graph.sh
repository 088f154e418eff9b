#!/bin/bash
# ViT-B/16 bf16 vs fp8, eager and hipGraph-captured, one box.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for g in 0 1; do
  for p in bf16 fp8; do
    timeout -k 10 300 python -u bench.py --model vit_b16 --precision $p --graph $g --steps 20 --warmup 5 > gpurun_out/vit_${p}_g$g.log 2>&1 || exit $?
    echo "$p graph=$g $(grep -o '"value": [0-9.]*, "unit": "[a-z/]*", "n_gpus": 1, "steps": 20, "warmup": 5, "ms_per_step": [0-9.]*' gpurun_out/vit_${p}_g$g.log)"
  done
done
