#!/bin/bash
# Round 5 (at): side-stream conv weight gradients (PDT_WGRAD_STREAM_M): bit-identity tests, then the 128/rank
# graphed step at several pixel thresholds.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_graph_gpu.py -q -x --timeout 300 --timeout-method thread > gpurun_out/t_at.log 2>&1; rc=$?
echo "graph tests rc=$rc"; tail -2 gpurun_out/t_at.log; grep -E "^E  |^FAILED" gpurun_out/t_at.log | head; [ $rc -eq 0 ] || exit $rc
for m in 0 30000 110000 1000000000 0; do
  PDT_WGRAD_STREAM_M=$m timeout -k 10 400 python -u bench.py --global-batch 128 --steps 30 --warmup 5 --graph 1 > gpurun_out/at_$m.log 2>&1; rc=$?
  echo "M<=$m rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/at_$m.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/at_$m.log)"; [ $rc -eq 0 ] || exit $rc
done
