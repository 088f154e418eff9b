#!/bin/bash
# Round 5 (h): 3x3 pipeline probes (layer-1 weight-stationary kernel: dead-row skip, compute-only, load-only)
# and the per-kind 3x3 table; 3x3 tests with the new default.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py tests/test_headline_shapes_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_h.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/t_h.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest "tests/test_conv1x1_bwd_fused_gpu.py::test_resnet50_grads_fused_vs_unfused" -q -s --timeout 200 --timeout-method thread > gpurun_out/t_h2.log 2>&1; rc=$?
echo "oracle test rc=$rc"; grep -E "fused vs fp32|passed|failed|Error" gpurun_out/t_h2.log | head -8; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/conv3x3_bench.py --opts 0,1,3,5 --only 64@56 > gpurun_out/c3_probe.txt 2>&1; rc=$?
cat gpurun_out/c3_probe.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/conv3x3_bench.py --opts 0,1 > gpurun_out/c3_table.txt 2>&1; rc=$?
cat gpurun_out/c3_table.txt; exit $rc
