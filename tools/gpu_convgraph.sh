#!/bin/bash
# Which MIOpen solvers break hipGraph replay? heuristic (benchmark=0) mode on the test's ResNet-18 shapes.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
export MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_HIP_GROUP_BWD_XDLOPS=0 MIOPEN_DEBUG_GROUP_CONV_IMPLICIT_GEMM_HIP_WRW_XDLOPS=0
echo "== r18s heuristic"; timeout -k 10 300 python tools/diag_conv_graph.py 8 0 r18s 2>&1 | grep -E "BAD|TOTAL|Error" || true
echo "== r18s benchmark"; timeout -k 10 300 python tools/diag_conv_graph.py 8 1 r18s 2>&1 | grep -E "BAD|TOTAL|Error" || true
echo "== r50 heuristic b256"; timeout -k 10 400 python tools/diag_conv_graph.py 256 0 r50 2>&1 | grep -E "BAD|TOTAL|Error" || true
echo "== r18s heuristic, logging"; MIOPEN_LOG_LEVEL=5 timeout -k 10 300 python tools/diag_conv_graph.py 8 0 r18s > gpurun_out/miolog.txt 2>&1 || true
grep -iE "solver|BAD" gpurun_out/miolog.txt | sort | uniq -c | sort -rn | head -60
exit 0
