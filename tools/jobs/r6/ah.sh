#!/bin/bash
# ResNet-50 1024/GPU: eager (bench default) vs hipGraph-captured step
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out/r6
for g in 0 1 0 1; do
  timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --graph $g > gpurun_out/r6/ah_graph_$g.log 2>&1 || exit 3
  echo "graph=$g b1024 $(grep -o '"value": [0-9.]*' gpurun_out/r6/ah_graph_$g.log)"
done
