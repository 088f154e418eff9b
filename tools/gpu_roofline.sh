#!/bin/bash
# Per-shape ResNet-50 roofline: BN (under a kernel trace, to split reduce vs apply) and convs.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/rl
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rl/bn -o bn -- python3 tools/r50_roofline.py --part bn > gpurun_out/rl/bn.log 2>&1 || exit $?
timeout -k 10 600 python3 tools/r50_roofline.py --part conv > gpurun_out/rl/conv.log 2>&1
