#!/bin/bash
# Round 5 (s): the reference's 128/rank point on one GPU: host overhead, eager, graphed, graphed profile.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/host_overhead.py --batch-size 128 > gpurun_out/host128.log 2>&1; echo "host rc=$?"; tail -6 gpurun_out/host128.log
timeout -k 10 300 python -u bench.py --global-batch 128 --steps 30 --warmup 5 > gpurun_out/strong128_eager.log 2>&1; echo "eager rc=$? $(grep -o '"value": [0-9.]*' gpurun_out/strong128_eager.log)"
timeout -k 10 400 python -u bench.py --global-batch 128 --steps 30 --warmup 5 --graph 1 > gpurun_out/strong128_graph.log 2>&1; rc=$?; echo "graph rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/strong128_graph.log)"; [ $rc -eq 0 ] || exit $rc
rm -rf /tmp/p128; mkdir -p /tmp/p128
timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --output-format csv -d /tmp/p128 -o run -- python3 bench.py --global-batch 128 --steps 5 --warmup 3 --graph 1 > gpurun_out/prof128.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python tools/prof_window.py /tmp/p128 gpurun_out/steady_resnet50_b128_graph timed 5 > /dev/null && head -1 gpurun_out/steady_resnet50_b128_graph.md
python tools/prof_categories.py gpurun_out/steady_resnet50_b128_graph_kernels.csv > gpurun_out/steady_resnet50_b128_graph_categories.md 2>/dev/null; cat gpurun_out/steady_resnet50_b128_graph_categories.md
head -30 gpurun_out/steady_resnet50_b128_graph.md | cut -c1-150
