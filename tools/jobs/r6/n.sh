#!/bin/bash
# z3 virtual on the APPLY-GEMM blocks only (PDT_Z3_VIRTUAL=2): test, then same-box A/B (with layer 2 on the APPLY GEMM too)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u -m pytest tests/test_bwd_alg_gpu.py -k "unwritten or ds_alg" -v -s --timeout 240 --timeout-method thread > gpurun_out/r6/n_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r6/n_tests.log | tail -8
[ $rc -le 1 ] || exit $rc
for cfg in 0:64 2:64 2:128 0:64 2:64 2:128; do
  v=${cfg%%:*}; k=${cfg##*:}
  PDT_Z3_VIRTUAL=$v PDT_BN_APPLY_GEMM_K=$k timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6/n_bench_${v}_$k.log 2>&1 || exit 3
  echo "z3_virtual=$v apply_gemm_k=$k $(grep -o '"value": [0-9.]*' gpurun_out/r6/n_bench_${v}_$k.log)"
done
