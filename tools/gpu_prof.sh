#!/bin/bash
# Graph-vs-eager tests + rocprofv3 kernel stats of eager ResNet-50 bench (ours and stock).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_graph_gpu.py -q > gpurun_out/pytest_graph.log 2>&1
rc=$?; echo "graph test rc=$rc"; grep -E "passed|failed|Error|Mismatch|difference" gpurun_out/pytest_graph.log | head -20
if [ $rc -gt 1 ]; then exit $rc; fi
export TMPDIR=/tmp
for impl in ours torch_ddp; do
  mkdir -p /tmp/prof_$impl
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d /tmp/prof_$impl -o run -- python3 bench.py --steps 5 --warmup 3 --graph 0 --impl $impl > gpurun_out/prof_$impl.log 2>&1
  rc=$?; echo "prof $impl rc=$rc"; tail -1 gpurun_out/prof_$impl.log
  if [ $rc -ne 0 ]; then exit $rc; fi
  find /tmp/prof_$impl -name "*kernel_stats.csv" -exec cp {} gpurun_out/kernel_stats_$impl.csv \;
done
ls -la gpurun_out
