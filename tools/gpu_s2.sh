#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_conv_gpu.py tests/test_models_gpu.py tests/test_profile_gate_gpu.py tests/test_graph_gpu.py -q -x --timeout 200 --timeout-method thread > gpurun_out/s2_tests.log 2>&1; rc=$?
tail -2 gpurun_out/s2_tests.log; [ $rc -eq 0 ] || exit $rc
run() { n=$1; shift; timeout -k 10 500 python -u bench.py "$@" > gpurun_out/s2_$n.log 2>&1; rc=$?
  echo "$n rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/s2_$n.log)"; [ $rc -ne 0 ] && tail -5 gpurun_out/s2_$n.log; return $rc; }
run on --steps 20 --warmup 5 || exit 1
PDT_CONV1X1_S2=0 run off --steps 20 --warmup 5 || exit 1
run on2 --steps 20 --warmup 5 || exit 1
PDT_CONV1X1_S2=0 run off2 --steps 20 --warmup 5 || exit 1
