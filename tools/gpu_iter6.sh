#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_fp8_gpu.py tests/test_graph_gpu.py -x -q -m gpu > gpurun_out/fp8t.txt 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/fp8t.txt
[ $rc -le 1 ] || exit $rc
SKIP_TESTS=1 MODELS=vit_b16 BENCH_ARGS="--precision fp8" TAG=_fp8 bash tools/gpu_prof3.sh
