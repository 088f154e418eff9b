#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests/test_models_gpu.py tests/test_graph_gpu.py tests/test_lenet_gpu.py -x -q -m gpu > gpurun_out/k7.txt 2>&1; rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/k7.txt
[ $rc -le 1 ] || exit $rc
for a in "--impl torch_ddp" "" "--graph 1"; do
  timeout -k 10 200 python bench.py --model lenet --steps 200 --warmup 20 $a 2>&1 | grep -E "metric|Error" || exit 1
done
timeout -k 10 300 python bench.py --model vit_b16 --precision fp8 --steps 20 --warmup 5 2>&1 | grep -E "metric|Error" || exit 1
