#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
rm -rf gpurun_out/miopen_cache; cp -r miopen_cache gpurun_out/miopen_cache
export PDT_MIOPEN_CACHE=$PWD/gpurun_out/miopen_cache
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/b_r50.log 2>&1 || exit 1
echo "ours $(grep -o '"value": [0-9.]*' gpurun_out/b_r50.log) $(grep -o 'warmup step 1/5 done at [0-9.]*' gpurun_out/b_r50.log)"
python -c "import torch" && timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --impl torch_ddp > gpurun_out/b_r50_torch.log 2>&1 || exit 1
echo "torch $(grep -o '"value": [0-9.]*' gpurun_out/b_r50_torch.log) $(grep -o 'warmup step 1/5 done at [0-9.]*' gpurun_out/b_r50_torch.log)"
