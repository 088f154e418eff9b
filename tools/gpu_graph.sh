#!/bin/bash
# hipGraph capture check with the capture-safe MIOpen solver set, then eager vs graph bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_graph_gpu.py -x -q -m gpu 2>&1 | tail -5 || exit 1
timeout -k 10 400 python tools/diag_graph.py --model resnet50 --batch 256 --size 224 || exit 1
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --graph 0 || exit 1
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --graph 1 || exit 1
