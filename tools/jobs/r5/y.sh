#!/bin/bash
# Round 5 (y): 128x64-tile fp8 casts: tests, ViT-B/16 bf16 vs fp8 same box, fp8 step profile.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_fp8_gpu.py -v --timeout 120 --timeout-method thread > gpurun_out/t_y1.log 2>&1; rc=$?
echo "fp8 tests rc=$rc"; tail -2 gpurun_out/t_y1.log; grep -E "^E  |^FAILED" gpurun_out/t_y1.log | head -20; [ $rc -eq 0 ] || exit $rc
run() {
  local tag=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/vit_$tag.log 2>&1; local rc=$?
  echo "$tag rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/vit_$tag.log)"; return $rc
}
for i in 1 2; do
  run bf16_$i python3 bench.py --model vit_b16 --steps 20 --warmup 5 || exit 1
  run fp8_$i python3 bench.py --model vit_b16 --precision fp8 --steps 20 --warmup 5 || exit 1
done
rm -rf /tmp/p_vit; mkdir -p /tmp/p_vit
timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --output-format csv -d /tmp/p_vit -o run -- python3 bench.py --model vit_b16 --precision fp8 --steps 5 --warmup 3 > gpurun_out/prof_vit.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python tools/prof_window.py /tmp/p_vit gpurun_out/steady_vit_b16_fp8 timed 5 > /dev/null && head -24 gpurun_out/steady_vit_b16_fp8.md
