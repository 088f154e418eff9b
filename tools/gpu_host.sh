#!/bin/bash
# Host-overhead probe + eager-vs-hipGraph ResNet-50 bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/host_overhead.py --steps 6 --warmup 4 > gpurun_out/host.log 2>&1
rc=$?; grep "\[host\]" gpurun_out/host.log; [ $rc -eq 0 ] || { tail -20 gpurun_out/host.log; exit $rc; }
timeout -k 10 400 python -u bench.py --steps 20 --warmup 6 --graph 1 > gpurun_out/bench_graph.log 2>&1
rc=$?; grep -E "metric|Error" gpurun_out/bench_graph.log | cut -c1-300; exit $rc
