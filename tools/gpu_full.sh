#!/bin/bash
# Full GPU tier (harvesting the MIOpen caches into gpurun_out) + attention microbench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
rm -rf gpurun_out/miopen_cache; cp -r miopen_cache gpurun_out/miopen_cache
export PDT_MIOPEN_CACHE=$PWD/gpurun_out/miopen_cache
timeout -k 10 200 python -u tools/attn_bench.py > gpurun_out/attn_bench.log 2>&1; rc=$?
cat gpurun_out/attn_bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
exit $rc
