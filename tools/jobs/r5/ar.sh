#!/bin/bash
# Round 5 (ar): gemm.hip 256 x 128 tiles for few-tile shapes: tests, standalone old vs new, vs hipBLASLt.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/t_ar1.log 2>&1; rc=$?
echo "gemm tests rc=$rc"; tail -1 gpurun_out/t_ar1.log; grep -E "^E  |^FAILED" gpurun_out/t_ar1.log | head; [ $rc -eq 0 ] || exit $rc
for b in old p0; do
  timeout -k 10 120 tools/convbench/gemmb_$b > gpurun_out/gemm_ar_$b.txt 2>&1; rc=$?
  echo "== $b"; grep -v amdgpu.ids gpurun_out/gemm_ar_$b.txt; [ $rc -eq 0 ] || exit $rc
done
for e in none bias gelu; do
  timeout -k 10 300 python3 tools/gemm_bench.py --epi $e > gpurun_out/gemm_ar_lib_$e.txt 2>&1; rc=$?
  grep -v amdgpu.ids gpurun_out/gemm_ar_lib_$e.txt | python3 -c "
import sys, json
for l in sys.stdin:
    if l.startswith('{'):
        d = json.loads(l); print(f\"$e {d['shape']:<10} ours {d['ours_us']:7.1f} lib {d['lib_us']:7.1f} speed {d['speedup']:.3f} err {d['rel_err']}\")
"; [ $rc -eq 0 ] || exit $rc
done
