#!/bin/bash
# What the driver runs at round end: smoke(), then bench.py under torchrun (N=1 here; 1-GPU box).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/rh_smoke.log 2>&1; rc=$?
echo "smoke rc=$rc $(tail -1 gpurun_out/rh_smoke.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/rh_bench.log 2>&1; rc=$?
echo "torchrun bench rc=$rc"; grep -E "warmup step 1/|metric" gpurun_out/rh_bench.log | cut -c1-400; exit $rc
