#!/bin/bash
# Multi-rank paths on a 1-GPU box: torchrun N=1 over RCCL; N=2 on one GPU over RCCL (may be
# rejected: duplicate GPU) and over gloo (exercises the DDP reducer with 2 ranks on GPU tensors).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
timeout -k 10 300 $TR --nproc-per-node 1 --master-port 29511 bench.py --gpus 1 --steps 5 --warmup 3 --batch-size 64 > gpurun_out/mr_n1.log 2>&1
rc=$?; echo "torchrun n1 nccl rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/mr_n1.log)"; [ $rc -ne 0 ] && tail -5 gpurun_out/mr_n1.log
timeout -k 10 300 $TR --nproc-per-node 2 --master-port 29512 bench.py --gpus 2 --steps 5 --warmup 3 --batch-size 64 --backend gloo > gpurun_out/mr_n2_gloo.log 2>&1
rc=$?; echo "torchrun n2 gloo rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/mr_n2_gloo.log) $(grep -o '"final_loss": [0-9.a-zA-Z]*' gpurun_out/mr_n2_gloo.log)"; [ $rc -ne 0 ] && tail -8 gpurun_out/mr_n2_gloo.log
timeout -k 10 180 $TR --nproc-per-node 2 --master-port 29513 bench.py --gpus 2 --steps 5 --warmup 3 --batch-size 64 > gpurun_out/mr_n2_nccl.log 2>&1
rc=$?; echo "torchrun n2 nccl(same gpu) rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/mr_n2_nccl.log)"; [ $rc -ne 0 ] && grep -iE "error|duplicate|invalid" gpurun_out/mr_n2_nccl.log | head -5
exit 0
