#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u -m pytest "tests/test_models_gpu.py::test_resnet50_fp32_native_matches_fp64_oracle" tests/test_amp_gpu.py tests/test_linear_splitk_gpu.py -v -s --timeout 240 --timeout-method thread > gpurun_out/r6/l_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed|^E  |median" gpurun_out/r6/l_tests.log | tail -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/oracle_negative_check.py > gpurun_out/r6/l_negative.log 2>&1; echo "negative rc=$?"; grep -E "clean|wrong" gpurun_out/r6/l_negative.log
