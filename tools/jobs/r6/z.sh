#!/bin/bash
# ALG with G's hi half only (PDT_ALG_GLO=0): tests, microbench, same-box A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out/r6
timeout -k 10 400 python -u -m pytest tests/test_bwd_alg_gpu.py -x -v -s --timeout 240 --timeout-method thread > gpurun_out/r6/z_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed|vs fp32" gpurun_out/r6/z_tests.log | tail -10
[ $rc -eq 0 ] || exit $rc
for v in 1 0 1 0; do
  PDT_ALG_GLO=$v timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r6/z_bench_$v.log 2>&1 || exit 3
  echo "glo=$v b1024 $(grep -o '"value": [0-9.]*' gpurun_out/r6/z_bench_$v.log)"
done
