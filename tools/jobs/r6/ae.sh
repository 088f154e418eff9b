#!/bin/bash
# one-launch column sums: tests (kernels, fp8, linear, transformer models, determinism) + transformer A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out/r6
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_fp8_gpu.py tests/test_linear_splitk_gpu.py tests/test_models_gpu.py tests/test_determinism_gpu.py tests/test_gemm_gpu.py -q --timeout 240 --timeout-method thread > gpurun_out/r6/ae_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r6/ae_tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
for v in 1 0 1 0; do
  for m in gpt2_medium vit_b16; do
    PDT_COLSUM_ONE_LAUNCH=$v timeout -k 10 300 python3 bench.py --model $m --steps 20 --warmup 5 > gpurun_out/r6/ae_${m}_$v.log 2>&1 || exit 3
    echo "one=$v $m $(grep -o '"value": [0-9.]*' gpurun_out/r6/ae_${m}_$v.log)"
  done
done
