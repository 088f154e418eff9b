#!/bin/bash
# Round 5 (av): our fp8 MFMA GEMM: numerics tests, then ours vs torch._scaled_mm (hipBLASLt) per shape.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_fp8_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/t_av.log 2>&1; rc=$?
echo "fp8 gemm tests rc=$rc"; tail -2 gpurun_out/t_av.log; grep -E "^E  |^FAILED" gpurun_out/t_av.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/gemm_fp8_bench.py > gpurun_out/gemm_fp8_av.txt 2>&1; rc=$?
grep '^{' gpurun_out/gemm_fp8_av.txt | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(f\"{d['shape']:<14} ours {d['ours_us']:7.1f} lib {d['lib_us']:7.1f} speed {d['speedup']:.3f} {d['ours_tflops']:7.1f} TF err {d['rel_err_vs_lib']}\")
"; exit $rc
