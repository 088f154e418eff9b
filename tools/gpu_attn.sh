#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/attn_bench.py > gpurun_out/attn_bench.log 2>&1; rc=$?
cat gpurun_out/attn_bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -k "attention" --timeout 120 --timeout-method thread > gpurun_out/pytest_attn.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_attn.log; exit $rc
