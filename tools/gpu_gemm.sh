#!/bin/bash
# Linear GEMM A/B (tools/gemm_bench.py) for each epilogue given as argument (default: bias gelu).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
for epi in ${@:-bias gelu}; do
  timeout -k 10 300 python3 tools/gemm_bench.py --epi $epi > gpurun_out/gemm_$epi.jsonl 2> gpurun_out/gemm_$epi.err
  rc=$?; cat gpurun_out/gemm_$epi.jsonl; [ $rc -eq 0 ] || { tail -20 gpurun_out/gemm_$epi.err; exit $rc; }
done
