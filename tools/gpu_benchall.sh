#!/bin/bash
# Headline + secondary north-star benches (ours and the stock-PyTorch baseline B0), then profiles.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
run() { n=$1; shift; timeout -k 10 400 python -u bench.py "$@" > gpurun_out/b_$n.log 2>&1; rc=$?
  echo "$n rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/b_$n.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/b_$n.log)"
  [ $rc -ne 0 ] && tail -5 gpurun_out/b_$n.log; return $rc; }
run r50_ours --steps 20 --warmup 5 || exit 1
run r50_torch --steps 20 --warmup 5 --impl torch_ddp || exit 1
run gpt_ours --model gpt2_medium --steps 10 --warmup 3 || exit 1
run gpt_torch --model gpt2_medium --steps 10 --warmup 3 --impl torch_ddp || exit 1
run vit_ours --model vit_b16 --steps 10 --warmup 3 || exit 1
run vit_fp8 --model vit_b16 --steps 10 --warmup 3 --precision fp8 || exit 1
run vit_torch --model vit_b16 --steps 10 --warmup 3 --impl torch_ddp || exit 1
run vit_accum --model vit_b16 --steps 10 --warmup 3 --grad-accum 4 || exit 1
run lenet_graph --model lenet --steps 200 --warmup 20 --graph 1 || exit 1
for m in resnet50 vit_b16 gpt2_medium; do
  rm -rf /tmp/p_$m; mkdir -p /tmp/p_$m
  timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --output-format csv -d /tmp/p_$m -o run -- python3 bench.py --model $m --steps 5 --warmup 3 > gpurun_out/prof_$m.log 2>&1
  rc=$?; echo "prof $m rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python tools/prof_window.py /tmp/p_$m gpurun_out/steady_$m timed 5 > /dev/null
  head -1 gpurun_out/steady_$m.md
done
