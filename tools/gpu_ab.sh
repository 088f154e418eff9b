#!/bin/bash
# In-process A/B of env switches on the ResNet-50 bench (tools/ab_env.py); CONFIGS overrides.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 ${TAB:-900} python -u tools/ab_env.py --reps ${REPS:-2} --configs ${CONFIGS} --steps ${STEPS:-10} --warmup 3 $BENCH_ARGS > gpurun_out/ab.log 2>&1
rc=$?; grep "\[ab\]" gpurun_out/ab.log; exit $rc
