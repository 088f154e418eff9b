#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r6
timeout -k 10 600 python -u -m pytest tests/test_amp_gpu.py tests/test_ddp_gpu.py::test_ddp_debug_mode_rccl_world1 tests/test_graph_collectives_gpu.py "tests/test_models_gpu.py::test_resnet50_frozen_bn3_keeps_conv1_branch_gradient" "tests/test_models_gpu.py::test_resnet50_fp32_native_matches_stock" -v --timeout 180 --timeout-method thread > gpurun_out/r6/a_tests.log 2>&1
echo "tests rc=$?"; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r6/a_tests.log | tail -30
timeout -k 10 300 python -u tools/diag_oracle_fp64.py > gpurun_out/r6/a_diag.log 2>&1; echo "diag rc=$?"; cat gpurun_out/r6/a_diag.log | tail -22
timeout -k 10 300 python -u tools/diag_oracle_fp64.py --hw 128 --n 16 > gpurun_out/r6/a_diag128.log 2>&1; echo "diag128 rc=$?"; tail -16 gpurun_out/r6/a_diag128.log
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6/a_bench.log 2>&1; echo "bench rc=$?"; grep metric gpurun_out/r6/a_bench.log
