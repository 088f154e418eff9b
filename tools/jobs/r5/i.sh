#!/bin/bash
# Round 5 (i): layer-1 3x3 pinned software pipeline (opt bit 3) tests + probes; fp32-oracle diagnostic.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py tests/test_headline_shapes_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_i.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/t_i.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/conv3x3_bench.py --opts 1,9,11,13,29,25 --only 64@56 > gpurun_out/c3_probe_i.txt 2>&1; rc=$?
cat gpurun_out/c3_probe_i.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/diag_oracle.py > gpurun_out/diag_oracle.txt 2>&1; rc=$?
cat gpurun_out/diag_oracle.txt; exit $rc
