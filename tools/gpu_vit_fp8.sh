#!/bin/bash
# ViT-B/16 bf16 vs fp8 on one box (driver command shape) + the fp8 / split-K Linear GPU tests.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fp8_gpu.py tests/test_linear_splitk_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fp8_test.log 2>&1
rc=$?; tail -2 gpurun_out/fp8_test.log; [ $rc -eq 0 ] || exit $rc
for p in bf16 fp8; do
  timeout -k 10 300 python -u bench.py --model vit_b16 --precision $p --steps 20 --warmup 5 > gpurun_out/vit_$p.log 2>&1 || exit $?
  grep -o '"value": [0-9.]*, "unit": "[a-z/]*", "n_gpus": 1, "steps": 20, "warmup": 5, "ms_per_step": [0-9.]*' gpurun_out/vit_$p.log
done
