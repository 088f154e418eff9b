#!/bin/bash
# hipGraph grad diagnosis + steady-state (timed-window) kernel profiles of ours vs stock.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python tools/diag_graph.py > gpurun_out/diag_graph.log 2>&1
rc=$?; echo "diag rc=$rc"; grep -E "deterministic|Error" gpurun_out/diag_graph.log | head -20
if [ $rc -ne 0 ]; then tail -20 gpurun_out/diag_graph.log; exit $rc; fi
for impl in ours torch_ddp; do
  rm -rf /tmp/p_$impl; mkdir -p /tmp/p_$impl
  timeout -k 10 500 rocprofv3 --kernel-trace --marker-trace --output-format csv -d /tmp/p_$impl -o run -- python3 bench.py --steps 5 --warmup 4 --graph 0 --impl $impl > gpurun_out/prof_$impl.log 2>&1
  rc=$?; echo "prof $impl rc=$rc"; grep metric gpurun_out/prof_$impl.log | cut -c1-200
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/prof_$impl.log; exit $rc; fi
  python tools/prof_window.py /tmp/p_$impl gpurun_out/steady_$impl timed 5 > /dev/null
  head -30 gpurun_out/steady_$impl.md
done
