#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out/r6
timeout -k 10 400 python -u -m pytest tests/test_amp_gpu.py -v --timeout 180 --timeout-method thread > gpurun_out/r6/b_tests.log 2>&1
echo "tests rc=$?"; grep -E "PASSED|FAILED|ERROR|passed|failed|^E  " gpurun_out/r6/b_tests.log | tail -30
for a in "--model resnet50 --res-scale 0.2" "--model resnet18" "--model resnet18 --res-scale 0.2" "--model resnet50 --hw 64 --n 32 --res-scale 0.2"; do
  timeout -k 10 300 python -u tools/diag_oracle_fp64.py $a > gpurun_out/r6/b_diag.log 2>&1 || { echo "diag $a failed"; tail -5 gpurun_out/r6/b_diag.log; exit 1; }
  grep -A6 "res_scale" gpurun_out/r6/b_diag.log
done
PC_CFGS="b1024:" bash tools/gpu_prof_calls.sh && cp gpurun_out/calls_b1024.md gpurun_out/r6/ && cp gpurun_out/steady_b1024.md gpurun_out/r6/
