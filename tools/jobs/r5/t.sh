#!/bin/bash
# Round 5 (t): stem weight gradient from the pooled gradient (PDT_STEM_POOL_WGRAD): tests, in-step A/B.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread -k "stem or maxpool" > gpurun_out/t_t1.log 2>&1; rc=$?
echo "stem tests rc=$rc"; tail -2 gpurun_out/t_t1.log; grep -E "^E  |Error" gpurun_out/t_t1.log | head -10; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/ab_env.py --reps 2 --configs "base:" "poolwg0:PDT_STEM_POOL_WGRAD=0" > gpurun_out/ab_stem_pool.txt 2>&1; rc=$?
grep "^\[ab\]" gpurun_out/ab_stem_pool.txt | tail -4; exit $rc
