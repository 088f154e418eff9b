#!/bin/bash
# matrix-core small GEMM of the ALG backward: tests, microbench, same-box A/B (b1024, b128 graphed)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out/r6
timeout -k 10 400 python -u -m pytest tests/test_bwd_alg_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r6/y_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r6/y_tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/alg_bench.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r6/y_algbench.log || exit 4
for v in 1 0 1 0; do
  PDT_ALG_SMALL_MFMA=$v timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r6/y_bench_$v.log 2>&1 || exit 3
  echo "mfma=$v b1024 $(grep -o '"value": [0-9.]*' gpurun_out/r6/y_bench_$v.log)"
done
for v in 1 0; do
  PDT_ALG_SMALL_MFMA=$v timeout -k 10 300 python3 bench.py --global-batch 128 --steps 30 --warmup 5 --graph 1 > gpurun_out/r6/y_b128_$v.log 2>&1 || exit 3
  echo "mfma=$v b128 graph $(grep -o '"value": [0-9.]*' gpurun_out/r6/y_b128_$v.log)"
done
