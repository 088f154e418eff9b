#!/bin/bash
# LayerNorm / transformer-model GPU tests, then the fused-add+LN A/B (tools/gpu_tx2.sh).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -q -x --timeout 120 --timeout-method thread -k "layernorm or gpt or vit" > gpurun_out/tx_tests.log 2>&1; rc=$?
tail -2 gpurun_out/tx_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_tx2.sh
