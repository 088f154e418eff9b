#!/bin/bash
# A/B of per-shape 1x1 decisions: dgrad shapes whose output feeds a BatchNorm backward (our GEMM
# then also takes that BN's reduction) flipped from hipBLASLt to our kernel.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
A="bwd_data,bf16,401408,512,128=ours"
B="bwd_data,bf16,401408,128,512=ours"
C="bwd_data,bf16,100352,256,1024=ours"
timeout -k 10 800 python -u tools/ab_env.py --reps 2 --configs 'table:' "ab:PDT_CONV1X1_OVERRIDE=$A+$B" "abc:PDT_CONV1X1_OVERRIDE=$A+$B+$C" "a:PDT_CONV1X1_OVERRIDE=$A" --steps 10 --warmup 3 > gpurun_out/ab_flip.log 2>&1
rc=$?; grep "\[ab\]" gpurun_out/ab_flip.log; exit $rc
