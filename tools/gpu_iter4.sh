#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py tests/test_graph_gpu.py tests/test_models_gpu.py -x -q -m gpu > gpurun_out/k4.txt 2>&1; rc=$?; echo "tests rc=$rc"; tail -12 gpurun_out/k4.txt
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 30 --warmup 5 2>&1 | grep metric || exit 1
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --graph 1 2>&1 | grep metric || exit 1
SKIP_TESTS=1 MODELS="resnet50" bash tools/gpu_prof3.sh
