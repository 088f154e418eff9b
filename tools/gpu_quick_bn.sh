#!/bin/bash
# BN kernel tests + headline bench (one GPU).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "batchnorm or bn_" --timeout 120 --timeout-method thread > gpurun_out/bn_tests.log 2>&1
rc=$?; tail -3 gpurun_out/bn_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_q.log 2>&1
rc=$?; grep metric gpurun_out/bench_q.log; exit $rc
