#!/bin/bash
# Round 5 (ay): where the 1x1 apply / accumulate epilogues' time goes: mask stores (32), all stores (1), MFMA (2).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
PDT_PROBES=0,32,1,2,0 timeout -k 10 300 python -u tools/conv1x1_probe.py > gpurun_out/c1_probe_ay.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/c1_probe_ay.txt; exit $rc
