#!/bin/bash
# Round 5 (q): 3x3 table at the bench batch, opt 41 (default) vs 105 (+ asm LDS DMA in the halo kernel).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/conv3x3_bench.py --opts 41,105 > gpurun_out/c3_q.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/c3_q.txt; exit $rc
