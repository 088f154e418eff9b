#!/bin/bash
# Split-K transformer weight gradients: tests, then in-process A/B on ViT-B/16 and GPT-2-medium.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_models_gpu.py tests/test_fp8_gpu.py tests/test_graph_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/linsk_tests.log 2>&1
rc=$?; tail -2 gpurun_out/linsk_tests.log; [ $rc -eq 0 ] || { grep -E "Error|error|assert|FAILED" gpurun_out/linsk_tests.log | head -20; exit $rc; }
for m in vit_b16 gpt2_medium; do
  timeout -k 10 600 python -u tools/ab_env.py --reps 2 --configs 'splitk:' 'mm:PDT_LINEAR_SPLITK=0' --model $m --steps 10 --warmup 3 > gpurun_out/ab_linsk_$m.log 2>&1
  rc=$?; echo $m; grep "\[ab\]" gpurun_out/ab_linsk_$m.log; [ $rc -eq 0 ] || exit $rc
done
