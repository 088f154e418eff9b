#!/bin/bash
# Round 5 (ae): persistent gemm.hip vs the one-tile version (same box) + tests.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/t_ae1.log 2>&1; rc=$?
echo "gemm tests rc=$rc"; tail -1 gpurun_out/t_ae1.log; [ $rc -eq 0 ] || exit $rc
for b in old p0 p3; do
  timeout -k 10 120 tools/convbench/gemmb_$b > gpurun_out/gemm_$b.txt 2>&1; rc=$?
  echo "== $b"; grep -v amdgpu.ids gpurun_out/gemm_$b.txt; [ $rc -eq 0 ] || exit $rc
done
