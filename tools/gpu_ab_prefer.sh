#!/bin/bash
# A/B: measured 1x1 table vs our GEMM preferred per direction (BN reduce passes saved by its epilogues).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 800 python -u tools/ab_env.py --reps 2 --configs 'table:' 'pref_dgrad:PDT_CONV1X1_PREFER=bwd_data' 'pref_fwd:PDT_CONV1X1_PREFER=fwd' 'pref_both:PDT_CONV1X1_PREFER=fwd,bwd_data' --steps 10 --warmup 3 > gpurun_out/ab_prefer.log 2>&1
rc=$?; grep "\[ab\]" gpurun_out/ab_prefer.log; exit $rc
