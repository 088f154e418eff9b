#!/bin/bash
# LeNet kernels, hipGraph solver diagnosis, graph training check, fp8 GEMM microbench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_lenet_gpu.py -x -q -m gpu > gpurun_out/lenet_tests.txt 2>&1; echo "lenet tests rc=$?"; tail -15 gpurun_out/lenet_tests.txt
timeout -k 10 200 python tools/fp8_bench.py > gpurun_out/fp8_bench.txt 2>&1; echo "fp8 rc=$?"; cat gpurun_out/fp8_bench.txt | tail -12
timeout -k 10 300 python tools/diag_graph.py --model resnet50 --batch 64 --size 224 --lr 0.1 --steps 8 2>&1 | tail -4
bash tools/gpu_convgraph.sh
SKIP_TESTS=1 MODELS="gpt2_medium vit_b16" bash tools/gpu_prof3.sh
