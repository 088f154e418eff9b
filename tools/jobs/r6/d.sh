#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u -m pytest tests/test_gap_bwd_gpu.py "tests/test_amp_gpu.py::test_amp_fp16_ddp_step_matches_fp32_oracle" -v -s --timeout 180 --timeout-method thread > gpurun_out/r6/d_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed|^E  |amp16 ours" gpurun_out/r6/d_tests.log | tail -20
[ $rc -le 1 ] || exit $rc
for a in 1 2; do
PDT_BWD_ALG=$a PC_CFGS="alg$a:" bash tools/gpu_prof_calls.sh || exit 1
cp gpurun_out/calls_alg$a.md gpurun_out/steady_alg$a.md gpurun_out/r6/
done
