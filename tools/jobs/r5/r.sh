#!/bin/bash
# Round 5 (r): 4-wave 3x3 weight gradient: bit-exactness vs the 8-wave kernel, A/B, bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_headline_shapes_gpu.py -x -q --timeout 120 --timeout-method thread -k wgrad > gpurun_out/t_r1.log 2>&1; rc=$?
echo "wgrad tests rc=$rc"; tail -2 gpurun_out/t_r1.log; grep -E "^E  |Error" gpurun_out/t_r1.log | head -10; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/conv3x3_bench.py --opts 41,1041 --only wgrad > gpurun_out/c3_r.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/c3_r.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r.log 2>&1; rc=$?
echo "bench rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/bench_r.log)"; exit $rc
