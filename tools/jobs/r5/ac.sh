#!/bin/bash
# Round 5 (ac): gemm.hip time split (probes: 1 no MFMA, 2 no DMA, 3 no epilogue) + vs hipBLASLt.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
for p in 0 1 2 3; do
  timeout -k 10 120 tools/convbench/gemmb_p$p > gpurun_out/gemm_probe$p.txt 2>&1; rc=$?
  grep -v amdgpu.ids gpurun_out/gemm_probe$p.txt; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python3 tools/gemm_bench.py --epi none > gpurun_out/gemm_vs_lib.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/gemm_vs_lib.txt | tail -10; exit $rc
