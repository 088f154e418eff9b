#!/bin/bash
# Round 5 (aq): watchdog drain before capture: graph tests + repeated graphed benches (ViT fp8, ResNet 128/rank).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_graph_gpu.py tests/test_graph_collectives_gpu.py -q --timeout 200 --timeout-method thread > gpurun_out/t_aq1.log 2>&1; rc=$?
echo "graph tests rc=$rc"; tail -1 gpurun_out/t_aq1.log; [ $rc -eq 0 ] || exit $rc
ok=0; bad=0
for i in 1 2 3 4; do
  timeout -k 10 300 python3 bench.py --model vit_b16 --precision fp8 --steps 10 --warmup 3 --graph 1 > gpurun_out/aq_vit_$i.log 2>&1; rc=$?
  echo "vit fp8 graph $i rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/aq_vit_$i.log)"
  if [ $rc -eq 0 ]; then ok=$((ok+1)); else bad=$((bad+1)); fi
done
timeout -k 10 400 python3 bench.py --global-batch 128 --steps 20 --warmup 5 --graph 1 > gpurun_out/aq_r50.log 2>&1; rc=$?
echo "resnet 128/rank graph rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/aq_r50.log)"
echo "vit graphed ok=$ok failed=$bad"
