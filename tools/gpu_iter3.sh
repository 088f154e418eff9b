#!/bin/bash
# kernel tests for the strip GELU/colsum kernels + linear, graph tests, transformer benches.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py tests/test_graph_gpu.py -x -q -m gpu > gpurun_out/k3.txt 2>&1; rc=$?; echo "tests rc=$rc"; tail -12 gpurun_out/k3.txt
[ $rc -le 1 ] || exit $rc
for m in gpt2_medium vit_b16; do
  timeout -k 10 300 python bench.py --model $m --steps 10 --warmup 3 2>&1 | grep metric || exit 1
done
SKIP_TESTS=1 MODELS="gpt2_medium vit_b16" bash tools/gpu_prof3.sh
