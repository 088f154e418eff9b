#!/bin/bash
# slice_sum kernel: tests, A/B on GPT-2-medium / ViT, then the batch-1024 ResNet-50 bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "slice_sum" --timeout 120 --timeout-method thread > gpurun_out/ss_tests.log 2>&1
rc=$?; tail -2 gpurun_out/ss_tests.log; [ $rc -eq 0 ] || { grep -E "Error|error|assert|FAILED" gpurun_out/ss_tests.log | head -20; exit $rc; }
for m in gpt2_medium vit_b16; do
  timeout -k 10 600 python -u tools/ab_env.py --reps 2 --configs 'kernel:' 'aten:PDT_SLICE_SUM=0' --model $m --steps 10 --warmup 3 > gpurun_out/ab_ss_$m.log 2>&1
  rc=$?; echo $m; grep "\[ab\]" gpurun_out/ab_ss_$m.log; [ $rc -eq 0 ] || exit $rc
done
SIZES=1024 bash tools/gpu_bsz.sh
