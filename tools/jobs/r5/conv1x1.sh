#!/bin/bash
# Round 5: the persistent 1x1 GEMM — new GPU tests, mode A/B timings, then the round's other new tests
# and the default bench (all steps time-limited, chained: the first failure ends the call).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_conv1x1_persist_gpu.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/t_persist.log 2>&1; rc=$?; echo "persist tests rc=$rc"; tail -12 gpurun_out/t_persist.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/conv1x1_persist_bench.py --rounds 3 > gpurun_out/persist_bench.txt 2>&1; rc=$?
echo "persist bench rc=$rc"; cat gpurun_out/persist_bench.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_p2p_gpu.py tests/test_graph_gpu.py tests/test_embedding_gpu.py \
  tests/test_conv1x1_ours_gpu.py -x -v --timeout 180 --timeout-method thread > gpurun_out/t_new.log 2>&1; rc=$?
echo "new tests rc=$rc"; tail -8 gpurun_out/t_new.log; [ $rc -eq 0 ] || exit $rc
for m in 0 1; do
  PDT_CONV1X1_PERSIST=$m timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_p$m.log 2>&1
  rc=$?; echo "bench persist=$m rc=$rc"; grep -E "metric" gpurun_out/bench_p$m.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
done
