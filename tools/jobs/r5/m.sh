#!/bin/bash
# Round 5 (m): row-tile 3x3 with precomputed fragment offsets: tests, A/B, probes; fp32-oracle diag + test.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_headline_shapes_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_m1.log 2>&1; rc=$?
echo "headline tests rc=$rc"; tail -2 gpurun_out/t_m1.log; grep -E "^E  |Error" gpurun_out/t_m1.log | head -10; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/conv3x3_bench.py --opts 9,41,43,45 --only 64@56 > gpurun_out/c3_m.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/c3_m.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/diag_oracle.py > gpurun_out/diag_oracle3.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/diag_oracle3.txt | tail -6; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest "tests/test_conv1x1_bwd_fused_gpu.py::test_resnet50_grads_fused_vs_unfused" -q -s --timeout 250 --timeout-method thread > gpurun_out/t_m2.log 2>&1; rc=$?
echo "oracle test rc=$rc"; grep -E "fused vs fp32|passed|failed|Error" gpurun_out/t_m2.log | head -6
exit 0
