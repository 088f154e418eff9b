#!/bin/bash
# Round 5 (n): fp32 native-vs-stock gradient diagnostic.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/diag_oracle.py > gpurun_out/diag_oracle4.txt 2>&1; rc=$?
grep -v "amdgpu.ids\|Warning\|detach\|return float" gpurun_out/diag_oracle4.txt | tail -20; exit $rc
