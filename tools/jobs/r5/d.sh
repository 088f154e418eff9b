#!/bin/bash
# Round 5 (d): in-process A/B of the 1x1-conv back-end preference (our GEMMs instead of hipBLASLt on the
# layer 3-4 shapes) + the BN finalize change, then the default bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_bn_tiles_gpu.py tests/test_determinism_gpu.py -x -q --timeout 200 \
  --timeout-method thread > gpurun_out/t_bn.log 2>&1; rc=$?; echo "bn tests rc=$rc"; tail -2 gpurun_out/t_bn.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u tools/ab_env.py --reps 2 --configs 'base:' 'ours_fd:PDT_CONV1X1_PREFER=fwd,bwd_data' \
  'ours_all:PDT_CONV1X1_PREFER=fwd,bwd_data,bwd_weight' --steps 20 --warmup 5 > gpurun_out/ab_r5d.txt 2>&1
rc=$?; echo "ab rc=$rc"; grep "\[ab\]" gpurun_out/ab_r5d.txt; exit $rc
