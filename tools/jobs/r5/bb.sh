#!/bin/bash
# Round 5 (bb): fp8 GEMM split-K for the weight-gradient shapes: fp8 + bf16 GEMM tests, then ours vs hipBLASLt
# (default heuristics and the TunableOp table).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_fp8_gpu.py tests/test_gemm_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/t_bb.log 2>&1; rc=$?
echo "gemm tests rc=$rc"; tail -2 gpurun_out/t_bb.log; grep -E "^E  |^FAILED" gpurun_out/t_bb.log | head; [ $rc -eq 0 ] || exit $rc
fmt() { python3 -c "
import sys, json
for l in sys.stdin:
    if l.startswith('{'):
        d = json.loads(l); print(f\"{d['shape']:<16} ours {d['ours_us']:7.1f} lib {d['lib_us']:7.1f} speed {d['speedup']:.3f} {d['ours_tflops']:7.1f} TF err {d['rel_err_vs_lib']}\")
"; }
timeout -k 10 300 python -u tools/gemm_fp8_bench.py > gpurun_out/gemm_fp8_bb.txt 2>&1; rc=$?
fmt < gpurun_out/gemm_fp8_bb.txt; [ $rc -eq 0 ] || { tail -5 gpurun_out/gemm_fp8_bb.txt; exit $rc; }
echo "== with the TunableOp table (lib = tuned hipBLASLt)"
mkdir -p /tmp/tt && cp tuning/tunableop_gfx950.csv /tmp/tt/t0.csv
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=/tmp/tt/t%d.csv SHAPES=vit_qkv_wgrad,vit_proj_wgrad,vit_fc1_wgrad,vit_fc2_wgrad,vit_qkv,vit_fc1 \
  timeout -k 10 300 python -u tools/gemm_fp8_bench.py > gpurun_out/gemm_fp8_bb_tuned.txt 2>&1; rc=$?
fmt < gpurun_out/gemm_fp8_bb_tuned.txt; exit $rc
