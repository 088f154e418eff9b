#!/bin/bash
# Round 5 (am): 128/rank (reference global-batch semantics at N=8) with the round's final kernels: graphed x2 + window.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 400 python -u bench.py --global-batch 128 --steps 30 --warmup 5 --graph 1 > gpurun_out/am_g$i.log 2>&1; rc=$?
  echo "graph $i rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/am_g$i.log)"; [ $rc -eq 0 ] || exit $rc
done
rm -rf /tmp/p128; mkdir -p /tmp/p128
timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --output-format csv -d /tmp/p128 -o run -- python3 bench.py --global-batch 128 --steps 10 --warmup 5 --graph 1 > gpurun_out/prof128.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python tools/prof_window.py /tmp/p128 gpurun_out/steady_resnet50_b128_graph timed 10 > /dev/null && head -1 gpurun_out/steady_resnet50_b128_graph.md
python tools/prof_categories.py gpurun_out/steady_resnet50_b128_graph_kernels.csv > gpurun_out/steady_resnet50_b128_graph_categories.md 2>/dev/null; tail -3 gpurun_out/steady_resnet50_b128_graph_categories.md
