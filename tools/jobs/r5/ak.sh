#!/bin/bash
# Round 5 (ak): GPT-2-medium bf16 vs fp8 same box x2 + fp8 step profile.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
run() {
  local tag=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/ak_$tag.log 2>&1; local rc=$?
  echo "$tag rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/ak_$tag.log)"; return $rc
}
for i in 1 2; do
  run gpt_bf16_$i python3 bench.py --model gpt2_medium --steps 10 --warmup 3 || exit 1
  run gpt_fp8_$i python3 bench.py --model gpt2_medium --precision fp8 --steps 10 --warmup 3 || exit 1
done
rm -rf /tmp/p_gpt; mkdir -p /tmp/p_gpt
timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --output-format csv -d /tmp/p_gpt -o run -- python3 bench.py --model gpt2_medium --precision fp8 --steps 5 --warmup 3 > gpurun_out/prof_gpt.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python tools/prof_window.py /tmp/p_gpt gpurun_out/steady_gpt2_medium_fp8 timed 5 > /dev/null && head -26 gpurun_out/steady_gpt2_medium_fp8.md
