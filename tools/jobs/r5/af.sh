#!/bin/bash
# Round 5 (af): fp8 weight-gradient token split on two streams: test + ViT / GPT-2 A/B.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fp8_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/t_af1.log 2>&1; rc=$?
echo "fp8 tests rc=$rc"; tail -1 gpurun_out/t_af1.log; grep -E "^E  |^FAILED" gpurun_out/t_af1.log | head; [ $rc -eq 0 ] || exit $rc
run() {
  local tag=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/af_$tag.log 2>&1; local rc=$?
  echo "$tag rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/af_$tag.log)"; return $rc
}
for i in 1 2; do
  run vit_s0_$i PDT_FP8_WGRAD_SPLIT=0 python3 bench.py --model vit_b16 --precision fp8 --steps 20 --warmup 5 || exit 1
  run vit_s1_$i PDT_FP8_WGRAD_SPLIT=1 python3 bench.py --model vit_b16 --precision fp8 --steps 20 --warmup 5 || exit 1
done
run vit_s0_g PDT_FP8_WGRAD_SPLIT=0 python3 bench.py --model vit_b16 --precision fp8 --steps 20 --warmup 5 --graph 1 || exit 1
run vit_s1_g PDT_FP8_WGRAD_SPLIT=1 python3 bench.py --model vit_b16 --precision fp8 --steps 20 --warmup 5 --graph 1 || exit 1
run gpt_s0 PDT_FP8_WGRAD_SPLIT=0 python3 bench.py --model gpt2_medium --precision fp8 --steps 10 --warmup 3 || exit 1
run gpt_s1 PDT_FP8_WGRAD_SPLIT=1 python3 bench.py --model gpt2_medium --precision fp8 --steps 10 --warmup 3 || exit 1
