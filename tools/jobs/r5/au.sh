#!/bin/bash
# Round 5 (au): BN tile finalize with 32 tiles per level-1 block + batched tail loads: BN / determinism / graph
# tests, then the 128/rank graphed step and the default 1024 step, 32 vs 128 tiles per block.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_bn_tiles_gpu.py tests/test_kernels_gpu.py tests/test_conv_gpu.py tests/test_conv_s2_gpu.py tests/test_conv1x1_bwd_fused_gpu.py tests/test_determinism_gpu.py tests/test_graph_gpu.py tests/test_headline_shapes_gpu.py -q -x --timeout 300 --timeout-method thread > gpurun_out/t_au.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/t_au.log; grep -E "^E  |^FAILED|ERROR" gpurun_out/t_au.log | head; [ $rc -eq 0 ] || exit $rc
for t in 128 32 128 32; do
  PDT_BN_TILES_PER_BLOCK=$t timeout -k 10 400 python -u bench.py --global-batch 128 --steps 30 --warmup 5 --graph 1 > gpurun_out/au_g_$t.log 2>&1; rc=$?
  echo "b128 graph tpb=$t rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/au_g_$t.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/au_g_$t.log)"; [ $rc -eq 0 ] || exit $rc
done
for t in 128 32; do
  PDT_BN_TILES_PER_BLOCK=$t timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/au_b_$t.log 2>&1; rc=$?
  echo "b1024 tpb=$t rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/au_b_$t.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/au_b_$t.log)"; [ $rc -eq 0 ] || exit $rc
done
