#!/bin/bash
# Round 5 (c): fused-backward headline test, in-process A/B (persistence, layer-2 fused backward), and a
# steady-state rocprofv3 window of the default bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv1x1_bwd_fused_gpu.py -x -q --timeout 200 --timeout-method thread \
  -k headline > gpurun_out/t_fused_head.log 2>&1; rc=$?; echo "fused headline rc=$rc"; tail -2 gpurun_out/t_fused_head.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/ab_env.py --reps 2 --configs 'base:' 'p0:PDT_CONV1X1_PERSIST=0' \
  'p2:PDT_CONV1X1_PERSIST=2' 'nf2:PDT_BWD_FUSED_SHAPES=256x64' --steps 20 --warmup 5 > gpurun_out/ab_r5c.txt 2>&1
rc=$?; echo "ab rc=$rc"; grep "\[ab\]" gpurun_out/ab_r5c.txt; [ $rc -eq 0 ] || exit $rc
rm -rf /tmp/p_r50; mkdir -p /tmp/p_r50
timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --output-format csv -d /tmp/p_r50 -o run -- python3 bench.py --steps 5 --warmup 3 > gpurun_out/prof_r50.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python tools/prof_window.py /tmp/p_r50 gpurun_out/steady_resnet50_b1024 timed 5 > /dev/null && head -3 gpurun_out/steady_resnet50_b1024.md
python tools/prof_categories.py gpurun_out/steady_resnet50_b1024_kernels.csv > gpurun_out/steady_resnet50_b1024_categories.md; cat gpurun_out/steady_resnet50_b1024_categories.md
