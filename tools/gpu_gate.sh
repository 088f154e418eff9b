#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_profile_gate_gpu.py tests/test_conv_gpu.py -v --timeout 200 --timeout-method thread > gpurun_out/gate.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|assert" gpurun_out/gate.log | head -30; tail -2 gpurun_out/gate.log; exit $rc
