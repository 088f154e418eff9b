#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out/r6
timeout -k 10 400 python -u tools/conv1x1_wgrad_bench.py --variants=-1,0,4 --wgs=0,512 --miopen 0 > gpurun_out/r6/i_wgrad_bench.txt 2>&1; echo "wgrad bench rc=$?"; cut -c1-60,200- gpurun_out/r6/i_wgrad_bench.txt | tail -12
for m in vit_b16 gpt2_medium; do
  for le in auto 0; do
  PDT_LINEAR_EPILOGUE=$le PDT_LINEAR_DUMP=gpurun_out/r6/linear_$m.json timeout -k 10 400 python3 bench.py --model $m --steps 10 --warmup 3 > gpurun_out/r6/i_bench_${m}_$le.log 2>&1 || { echo "$m failed"; tail -5 gpurun_out/r6/i_bench_${m}_$le.log; exit 1; }
  echo "$m linear=$le $(grep -o '"value": [0-9.]*' gpurun_out/r6/i_bench_${m}_$le.log)"
  done
done
cat gpurun_out/r6/linear_*.json
