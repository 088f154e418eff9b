#!/bin/bash
# bf16 bias in the GELU kernels: tests + transformer bench (GPT-2 medium / ViT-B/16 bf16)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k gelu tests/test_fp8_gpu.py tests/test_models_gpu.py -q --timeout 240 --timeout-method thread > gpurun_out/r6/ad_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r6/ad_tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
for m in gpt2_medium vit_b16; do
  timeout -k 10 300 python3 bench.py --model $m --steps 20 --warmup 5 > gpurun_out/r6/ad_$m.log 2>&1 || exit 3
  echo "$m $(grep -o '"value": [0-9.]*' gpurun_out/r6/ad_$m.log)"
done
