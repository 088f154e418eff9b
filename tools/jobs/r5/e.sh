#!/bin/bash
# Round 5 (e): BN finalize tests; conv1x1 tile/persistence microbench (incl. conv1's dgrad); in-process A/B of
# the 1x1 back-end preference; then the kernel-coverage gate of the GPU tier.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_bn_tiles_gpu.py tests/test_determinism_gpu.py -x -q --timeout 200 \
  --timeout-method thread > gpurun_out/t_bn.log 2>&1; rc=$?; echo "bn tests rc=$rc"; tail -2 gpurun_out/t_bn.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/conv1x1_persist_bench.py --rounds 3 --modes 0,w,1 > gpurun_out/c1x1_bench_e.txt 2>&1
rc=$?; echo "c1x1 bench rc=$rc"; cat gpurun_out/c1x1_bench_e.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/ab_env.py --reps 2 --configs 'base:' 'ours_fd:PDT_CONV1X1_PREFER=fwd,bwd_data' \
  'ours_all:PDT_CONV1X1_PREFER=fwd,bwd_data,bwd_weight' 'gapply128:PDT_BN_APPLY_GEMM_K=128' 'defer2:PDT_BN2_DEFER=1' --steps 20 --warmup 5 > gpurun_out/ab_r5e.txt 2>&1
rc=$?; echo "ab rc=$rc"; grep "\[ab\]" gpurun_out/ab_r5e.txt; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_coverage.sh
