#!/bin/bash
# Round 5 (an): split-K depth of our weight gradients at 128/rank and 1024/GPU.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/wgrad_target_sweep.py --batch 128 > gpurun_out/wgrad_sweep_128.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/wgrad_sweep_128.txt
timeout -k 10 300 python3 tools/wgrad_target_sweep.py --batch 1024 --targets 0,128,192,256,384 --rounds 2 > gpurun_out/wgrad_sweep_1024.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/wgrad_sweep_1024.txt
