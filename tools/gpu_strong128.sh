#!/bin/bash
# Reference global-batch semantics at the 8-GPU point (train.py:82: ceil(1024/8) = 128 per rank),
# rehearsed on one GPU: host overhead per step, eager vs hipGraph-captured step.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/host_overhead.py --batch-size 128 > gpurun_out/host128.log 2>&1; echo "host rc=$?"; tail -4 gpurun_out/host128.log
timeout -k 10 300 python -u bench.py --global-batch 128 --steps 30 --warmup 5 --graph 0 > gpurun_out/strong128_eager.log 2>&1; echo "eager rc=$?"; grep -o '"value": [0-9.]*, "unit": "[a-z/]*", "n_gpus": 1, "steps": 30, "warmup": 5, "ms_per_step": [0-9.]*\|"final_loss": [^}]*' gpurun_out/strong128_eager.log
timeout -k 10 400 python -u bench.py --global-batch 128 --steps 30 --warmup 5 --graph 1 > gpurun_out/strong128_graph.log 2>&1; echo "graph rc=$?"; grep -o '"value": [0-9.]*, "unit": "[a-z/]*", "n_gpus": 1, "steps": 30, "warmup": 5, "ms_per_step": [0-9.]*\|"final_loss": [^}]*' gpurun_out/strong128_graph.log
