#!/bin/bash
# downsample ALG (PDT_DS_ALG): tests, then same-box A/B of the bench at 0 / 512 / 2048
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out/r6
timeout -k 10 600 python -u -m pytest tests/test_bwd_alg_gpu.py -k "resnet50 or determin" tests/test_conv1x1_bwd_fused_gpu.py tests/test_determinism_gpu.py -v -s --timeout 240 --timeout-method thread > gpurun_out/r6/m_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed|vs fp32" gpurun_out/r6/m_tests.log | tail -16
[ $rc -le 1 ] || exit $rc
for v in 0 512 2048 0 512; do
  PDT_DS_ALG=$v timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6/m_bench_$v.log 2>&1 || exit 3
  echo "ds_alg=$v $(grep -o '"value": [0-9.]*' gpurun_out/r6/m_bench_$v.log)"
done
