#!/bin/bash
# Round 5 (k): layer-1 row-tile 3x3 kernel + VALU cross-lane reductions: new tests first, full GPU tier,
# 3x3 A/B (opt 9 = old weight-stationary, 41 = row tiles), bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_headline_shapes_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_k1.log 2>&1; rc=$?
echo "headline tests rc=$rc"; tail -3 gpurun_out/t_k1.log; grep -E "^E  |Error" gpurun_out/t_k1.log | head -10; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/conv3x3_bench.py --opts 9,41 --only 64@56 > gpurun_out/c3_k.txt 2>&1; rc=$?
cat gpurun_out/c3_k.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_k.log 2>&1; rc=$?
echo "bench rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/bench_k.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_k_all.log 2>&1; rc=$?
echo "gpu tier rc=$rc"; tail -3 gpurun_out/t_k_all.log; grep -E "^FAILED|^E  " gpurun_out/t_k_all.log | head -10
exit $rc
