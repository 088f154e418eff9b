#!/bin/bash
# ResNet head on the colsum Linear: graph replay after churn at 1024/GPU, then the default (graphed) bench twice + eager
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out/r6
timeout -k 10 300 python3 -u tools/diag_graph_model.py --batch-size 1024 > gpurun_out/r6/am_diag.log 2>&1 || { echo "diag rc=$?"; exit 5; }
grep "^replay\|^  fc.bias " gpurun_out/r6/am_diag.log; grep -A3 "^replay 1" gpurun_out/r6/am_diag.log
timeout -k 10 100 python3 -u tools/diag_graph_colsum_bwd.py > gpurun_out/r6/am_colsum_bwd.log 2>&1 || exit 6
for i in 1 2; do
  timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6/am_bench_$i.log 2>&1 || exit 3
  echo "default bench $i: $(grep -o '"value": [0-9.]*' gpurun_out/r6/am_bench_$i.log) $(grep -o '"graph": [a-z]*' gpurun_out/r6/am_bench_$i.log) $(grep -o '"final_loss": [^}]*' gpurun_out/r6/am_bench_$i.log)"
done
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --graph 0 > gpurun_out/r6/am_bench_eager.log 2>&1 || exit 3
echo "eager: $(grep -o '"value": [0-9.]*' gpurun_out/r6/am_bench_eager.log) $(grep -o '"final_loss": [^}]*' gpurun_out/r6/am_bench_eager.log)"
