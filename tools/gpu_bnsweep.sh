#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/bn_reduce_sweep.py > gpurun_out/bnsweep.log 2>&1; rc=$?
cat gpurun_out/bnsweep.log | grep -v amdgpu.ids; exit $rc
