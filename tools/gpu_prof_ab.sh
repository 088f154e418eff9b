#!/bin/bash
# Kernel-trace A/B of two env configurations in ONE process (tools/ab_env.py), windows split by
# occurrence of the "timed" range, then a per-kernel diff. CONFIGS="a:VAR=v b:VAR=v".
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf /tmp/p_ab; mkdir -p /tmp/p_ab
timeout -k 10 600 rocprofv3 --kernel-trace --marker-trace --output-format csv -d /tmp/p_ab -o run -- python3 tools/ab_env.py --reps 1 --configs ${CONFIGS} --steps 5 --warmup 3 $BENCH_ARGS > gpurun_out/prof_ab.log 2>&1
rc=$?; grep "\[ab\]" gpurun_out/prof_ab.log; [ $rc -eq 0 ] || exit $rc
python tools/prof_window.py /tmp/p_ab gpurun_out/ab_A timed 5 0 > /dev/null
python tools/prof_window.py /tmp/p_ab gpurun_out/ab_B timed 5 1 > /dev/null
python tools/prof_diff.py gpurun_out/ab_A_kernels.csv gpurun_out/ab_B_kernels.csv 5 45 > gpurun_out/ab_diff.md
head -50 gpurun_out/ab_diff.md
