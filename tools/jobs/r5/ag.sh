#!/bin/bash
# Round 5 (ag): fp8 producer kernels (bias in LDS, occupancy-sized grids): tests + per-kernel bandwidth.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fp8_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/t_ag1.log 2>&1; rc=$?
echo "fp8 tests rc=$rc"; tail -1 gpurun_out/t_ag1.log; grep -E "^E  |^FAILED" gpurun_out/t_ag1.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 tools/fp8_cast_bench.py > gpurun_out/fp8_cast_bench.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/fp8_cast_bench.txt; exit $rc
