#!/bin/bash
# same box: eager ResNet-50 1024/GPU with the colsum head vs aten's nn.Linear head, then graphed (colsum head)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out/r6
for h in 1 0 1 0; do
  PDT_HEAD_COLSUM=$h timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --graph 0 > gpurun_out/r6/an_head$h.log 2>&1 || exit 3
  echo "eager head_colsum=$h $(grep -o '"value": [0-9.]*' gpurun_out/r6/an_head$h.log) $(grep -o '"final_loss": [^}]*' gpurun_out/r6/an_head$h.log)"
done
for i in 1 2; do
  timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r6/an_graph.log 2>&1 || exit 3
  echo "graph $(grep -o '"value": [0-9.]*' gpurun_out/r6/an_graph.log) $(grep -o '"final_loss": [^}]*' gpurun_out/r6/an_graph.log)"
done
