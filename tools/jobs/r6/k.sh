#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out/r6
for env in "X=1" "PDT_CONV1X1=miopen" "PDT_CONV1X1=gemm" "PDT_WGRAD_SPLITK=0" "PDT_CONV1X1_S2=0" "PDT_CONV3X3=miopen"; do
  env $env timeout -k 10 200 python -u tools/diag_oracle_fp64.py --res-scale 0.2 > gpurun_out/r6/k_diag.log 2>&1 || { echo "fail $env"; tail -3 gpurun_out/r6/k_diag.log; exit 1; }
  echo "== $env"; grep -E "native fp32 vs fp64|stock fp32 vs fp64" gpurun_out/r6/k_diag.log
done
