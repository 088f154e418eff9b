#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
echo "== default"; timeout -k 10 400 python tools/diag_conv_graph.py 64 2>&1 | grep -E "BAD|TOTAL|Error"
echo "== no asm GTC NHWC"; MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0 MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0 MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_FWD_GTC_XDLOPS_NHWC=0 timeout -k 10 400 python tools/diag_conv_graph.py 64 2>&1 | grep -E "BAD|TOTAL|Error"
echo "== no CK group bwd/wrw"; MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_HIP_GROUP_BWD_XDLOPS=0 MIOPEN_DEBUG_GROUP_CONV_IMPLICIT_GEMM_HIP_WRW_XDLOPS=0 timeout -k 10 400 python tools/diag_conv_graph.py 64 2>&1 | grep -E "BAD|TOTAL|Error"
exit 0
