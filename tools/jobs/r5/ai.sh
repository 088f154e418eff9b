#!/bin/bash
# Round 5 (ai): striped amax rows: producer bandwidth, ViT-B/16 / GPT-2 bf16 vs fp8 same box, fp8 profile.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/fp8_cast_bench.py > gpurun_out/fp8_cast_bench.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/fp8_cast_bench.txt
run() {
  local tag=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/ai_$tag.log 2>&1; local rc=$?
  echo "$tag rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/ai_$tag.log)"; return $rc
}
for i in 1 2; do
  run vit_bf16_$i python3 bench.py --model vit_b16 --steps 20 --warmup 5 || exit 1
  run vit_fp8_$i python3 bench.py --model vit_b16 --precision fp8 --steps 20 --warmup 5 || exit 1
done
run vit_bf16_g python3 bench.py --model vit_b16 --steps 20 --warmup 5 --graph 1 || exit 1
run vit_fp8_g python3 bench.py --model vit_b16 --precision fp8 --steps 20 --warmup 5 --graph 1 || exit 1
run gpt_bf16 python3 bench.py --model gpt2_medium --steps 10 --warmup 3 || exit 1
run gpt_fp8 python3 bench.py --model gpt2_medium --precision fp8 --steps 10 --warmup 3 || exit 1
rm -rf /tmp/p_vit; mkdir -p /tmp/p_vit
timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --output-format csv -d /tmp/p_vit -o run -- python3 bench.py --model vit_b16 --precision fp8 --steps 5 --warmup 3 > gpurun_out/prof_vit.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python tools/prof_window.py /tmp/p_vit gpurun_out/steady_vit_b16_fp8 timed 5 > /dev/null && head -22 gpurun_out/steady_vit_b16_fp8.md
