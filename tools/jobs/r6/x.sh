#!/bin/bash
# subsample side output (PDT_SUB_OUT): tests, then same-box A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u -m pytest tests/test_subsample_out_gpu.py tests/test_conv1x1_ours_gpu.py -x -v --timeout 240 --timeout-method thread > gpurun_out/r6/x_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r6/x_tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
for v in 1 0 1 0; do
  PDT_SUB_OUT=$v timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r6/x_bench_$v.log 2>&1 || exit 3
  echo "sub_out=$v $(grep -o '"value": [0-9.]*' gpurun_out/r6/x_bench_$v.log)"
done
