#!/bin/bash
# Round 5 (ad): persistent gemm.hip (epilogue overlapped with the next tile's first K-steps): tests, probes, vs hipBLASLt.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/t_ad1.log 2>&1; rc=$?
echo "gemm tests rc=$rc"; tail -2 gpurun_out/t_ad1.log; grep -E "^E  |^FAILED" gpurun_out/t_ad1.log | head -20; [ $rc -eq 0 ] || exit $rc
for p in 0 3; do
  timeout -k 10 120 tools/convbench/gemmb_p$p > gpurun_out/gemm_probe$p.txt 2>&1; rc=$?
  grep -v amdgpu.ids gpurun_out/gemm_probe$p.txt; [ $rc -eq 0 ] || exit $rc
done
for e in none bias gelu; do
  timeout -k 10 300 python3 tools/gemm_bench.py --epi $e > gpurun_out/gemm_vs_lib_$e.txt 2>&1; rc=$?
  grep -v amdgpu.ids gpurun_out/gemm_vs_lib_$e.txt | python3 -c "
import sys, json
for l in sys.stdin:
    if l.startswith('{'):
        d = json.loads(l); print(f\"$e {d['shape']:<10} ours {d['ours_us']:7.1f} lib {d['lib_us']:7.1f} speed {d['speedup']:.3f} err {d['rel_err']}\")
"; [ $rc -eq 0 ] || exit $rc
done
