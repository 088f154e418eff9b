#!/bin/bash
# Iteration run: GPU tests, bench variants, steady-state profile of ours.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/ -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -15 gpurun_out/pytest_gpu.log | grep -E "passed|failed|Error|assert" | head
if [ $rc -gt 1 ]; then exit $rc; fi
run() { # name args...
  n=$1; shift
  timeout -k 10 400 python bench.py "$@" > gpurun_out/b_$n.log 2>&1
  rc=$?; echo "$n rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/b_$n.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/b_$n.log) $(grep -o '"final_loss": [-0-9.a-zA-Z]*' gpurun_out/b_$n.log)"
  return $rc
}
run ours_eager --steps 20 --warmup 5 --graph 0 --deterministic 0 || exit 1
run ours_eager_det --steps 20 --warmup 5 --graph 0 --deterministic 1 || exit 1
run ours_graph --steps 20 --warmup 5 --graph 1 || exit 1
run torch_ddp --steps 20 --warmup 5 --impl torch_ddp || exit 1
rm -rf /tmp/p_ours; mkdir -p /tmp/p_ours
timeout -k 10 500 rocprofv3 --kernel-trace --marker-trace --output-format csv -d /tmp/p_ours -o run -- python3 bench.py --steps 5 --warmup 4 --graph 0 --deterministic 0 > gpurun_out/prof_ours.log 2>&1
rc=$?; echo "prof rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
python tools/prof_window.py /tmp/p_ours gpurun_out/steady_ours timed 5 > /dev/null
head -24 gpurun_out/steady_ours.md
