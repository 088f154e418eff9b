#!/bin/bash
# A/B: MIOpen's atomic-accumulate GTC NHWC bwd/wrw solvers (need zero-fill + cast passes) vs
# excluding them (CK / other solvers picked by find instead). Fresh find-db for the B arm.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/ab_base.log 2>&1 || exit 1
echo "base $(grep -o '"value": [0-9.]*' gpurun_out/ab_base.log)"
rm -rf gpurun_out/miopen_nogtc
export PDT_MIOPEN_CACHE=$PWD/gpurun_out/miopen_nogtc
export MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0 MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > gpurun_out/ab_nogtc.log 2>&1 || exit 1
echo "nogtc $(grep -o '"value": [0-9.]*' gpurun_out/ab_nogtc.log) $(grep -o 'warmup step 1/5 done at [0-9.]*' gpurun_out/ab_nogtc.log)"
