#!/bin/bash
# ViT-B/16 with gradient accumulation (BASELINE config 3): eager vs hipGraph-captured step.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for a in "--batch-size 512 --grad-accum 4" "--batch-size 512 --grad-accum 4 --graph 1" "--batch-size 512 --grad-accum 4 --graph 1 --precision fp8" "--grad-accum 4 --graph 1"; do
  timeout -k 10 300 python -u bench.py --model vit_b16 --steps 10 --warmup 4 $a > gpurun_out/vit.log 2>&1 || { echo "FAIL $a"; tail -5 gpurun_out/vit.log; exit 1; }
  echo "$a: $(grep -o '"value": [0-9.]*, "unit": "[a-z/]*"' gpurun_out/vit.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/vit.log)"
done
