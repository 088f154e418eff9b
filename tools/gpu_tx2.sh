#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
run() { n=$1; shift; timeout -k 10 400 python -u bench.py "$@" > gpurun_out/b_$n.log 2>&1; rc=$?
  echo "$n rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/b_$n.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/b_$n.log)"
  [ $rc -ne 0 ] && tail -5 gpurun_out/b_$n.log; return $rc; }
run gpt_fused --model gpt2_medium --steps 10 --warmup 3 || exit 1
PDT_FUSED_ADDLN=0 run gpt_unfused --model gpt2_medium --steps 10 --warmup 3 || exit 1
run gpt_fused2 --model gpt2_medium --steps 10 --warmup 3 || exit 1
PDT_FUSED_ADDLN=0 run gpt_unfused2 --model gpt2_medium --steps 10 --warmup 3 || exit 1
rm -rf /tmp/p_g; mkdir -p /tmp/p_g
timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --output-format csv -d /tmp/p_g -o run -- python3 bench.py --model gpt2_medium --steps 5 --warmup 3 > gpurun_out/prof_g.log 2>&1 || exit 1
python tools/prof_window.py /tmp/p_g gpurun_out/steady_gpt2_fused timed 5 > /dev/null
head -25 gpurun_out/steady_gpt2_fused.md | cut -c1-140
