#!/bin/bash
# Fresh-box verification exactly as the round-end driver runs it: headline bench (committed
# in-tree MIOpen find-db / GEMM tables, no PDT_MIOPEN_CACHE override), full GPU test tier, smoke.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
PDT_STACK_DUMP=60 timeout -k 10 ${TB:-300} python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_default.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -E "warmup|metric" gpurun_out/bench_default.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 ${TP:-600} python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
prc=$?; echo "pytest rc=$prc"; tail -15 gpurun_out/pytest_gpu.log
# rc 1 = some tests failed: still run smoke (GPU is healthy), but the script fails at the end
[ $prc -le 1 ] || exit $prc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
exit $prc
