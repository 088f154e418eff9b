#!/bin/bash
# ALG pixel threshold: tests, then b128 graphed + b1024 with threshold 50176 vs 0
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u -m pytest tests/test_bwd_alg_gpu.py -k "threshold or ds_alg" -v -s --timeout 240 --timeout-method thread > gpurun_out/r6/o_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r6/o_tests.log | tail -8
[ $rc -le 1 ] || exit $rc
for m in 0 50176 0 50176; do
  PDT_BWD_ALG_MIN_M=$m timeout -k 10 300 python3 bench.py --global-batch 128 --steps 30 --warmup 5 --graph 1 > gpurun_out/r6/o_b128_$m.log 2>&1 || exit 3
  echo "b128 graph min_m=$m $(grep -o '"value": [0-9.]*' gpurun_out/r6/o_b128_$m.log)"
done
for m in 0 50176; do
  PDT_BWD_ALG_MIN_M=$m timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r6/o_b1024_$m.log 2>&1 || exit 3
  echo "b1024 min_m=$m $(grep -o '"value": [0-9.]*' gpurun_out/r6/o_b1024_$m.log)"
done
