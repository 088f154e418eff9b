#!/bin/bash
# Round 5 (aj): rest of job ai (graphed ViT fp8, GPT-2 bf16 vs fp8, ViT fp8 profile).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
run() {
  local tag=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/ai_$tag.log 2>&1; local rc=$?
  echo "$tag rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/ai_$tag.log)"; return $rc
}
run gpt_bf16 python3 bench.py --model gpt2_medium --steps 10 --warmup 3 || exit 1
run gpt_fp8 python3 bench.py --model gpt2_medium --precision fp8 --steps 10 --warmup 3 || exit 1
rm -rf /tmp/p_vit; mkdir -p /tmp/p_vit
timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --output-format csv -d /tmp/p_vit -o run -- python3 bench.py --model vit_b16 --precision fp8 --steps 5 --warmup 3 > gpurun_out/prof_vit.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python tools/prof_window.py /tmp/p_vit gpurun_out/steady_vit_b16_fp8 timed 5 > /dev/null && head -22 gpurun_out/steady_vit_b16_fp8.md
run vit_fp8_g python3 bench.py --model vit_b16 --precision fp8 --steps 20 --warmup 5 --graph 1
