#!/bin/bash
# Round 5 (w): 3x3 weight gradient with precomputed swizzled tap offsets + compile-time pitch: tests, table, bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_conv_gpu.py tests/test_conv_s2_gpu.py tests/test_headline_shapes_gpu.py tests/test_conv1x1_ours_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/t_w1.log 2>&1; rc=$?
echo "conv tests rc=$rc"; tail -2 gpurun_out/t_w1.log; grep -E "^E  |^FAILED" gpurun_out/t_w1.log | head -10; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u tools/conv3x3_bench.py --opts 41 --only wgrad > gpurun_out/c3_w.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/c3_w.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_w.log 2>&1; rc=$?
echo "bench rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/bench_w.log)"; exit $rc
