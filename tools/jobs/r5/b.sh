#!/bin/bash
# Round 5 (b): fused-backward lockstep tests + slack A/B, the conv1x1 tests, the round's other new GPU tests,
# then the default bench (persistence default) — every step time-limited and chained.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_conv1x1_bwd_fused_gpu.py tests/test_conv1x1_persist_gpu.py -x -v \
  --timeout 300 --timeout-method thread > gpurun_out/t_fused.log 2>&1; rc=$?; echo "fused+persist tests rc=$rc"
tail -6 gpurun_out/t_fused.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bwd_fused_bench.py --layer 2 --rounds 3 --slacks 0,1,2,3,4 > gpurun_out/fused_slack_l2.txt 2>&1
rc=$?; echo "slack bench rc=$rc"; cat gpurun_out/fused_slack_l2.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_p2p_gpu.py tests/test_graph_gpu.py tests/test_embedding_gpu.py \
  tests/test_conv1x1_ours_gpu.py -x -v --timeout 180 --timeout-method thread > gpurun_out/t_new.log 2>&1; rc=$?
echo "new tests rc=$rc"; tail -4 gpurun_out/t_new.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_def.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -E "metric" gpurun_out/bench_def.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc
PDT_CONV1X1_PERSIST=0 timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_p0.log 2>&1
rc=$?; echo "bench p0 rc=$rc"; grep -oE '"value": [0-9.]+' gpurun_out/bench_p0.log; exit $rc
