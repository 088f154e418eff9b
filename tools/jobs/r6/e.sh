#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u -m pytest tests/test_bwd_alg_gpu.py tests/test_gap_bwd_gpu.py -v --timeout 180 --timeout-method thread > gpurun_out/r6/e_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed|^E  " gpurun_out/r6/e_tests.log | tail -20
[ $rc -le 1 ] || exit $rc
for a in 2 0 2; do
PDT_BWD_ALG=$a timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6/e_bench_alg$a.log 2>&1 || exit 1; echo "bench alg=$a $(grep -o '"value": [0-9.]*' gpurun_out/r6/e_bench_alg$a.log)"
done
PDT_BWD_ALG=2 PC_CFGS="alg2c:" bash tools/gpu_prof_calls.sh || exit 1
cp gpurun_out/calls_alg2c.md gpurun_out/steady_alg2c.md gpurun_out/r6/
