#!/bin/bash
# conv3x3 halo kernel with its LDS DMA through inline asm (PDT_CONV3X3_OPT bit 6: 41 -> 105): microbench + bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out/r6
for o in 41 105 41 105; do
  PDT_CONV3X3_OPT=$o timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r6/ac_bench_$o.log 2>&1 || exit 3
  echo "opt=$o b1024 $(grep -o '"value": [0-9.]*' gpurun_out/r6/ac_bench_$o.log)"
done
