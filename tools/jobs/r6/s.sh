#!/bin/bash
# the driver's order: GPU test tier, smoke, bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out/r6
timeout -k 10 1000 python -u -m pytest tests/ -q -m gpu --timeout 180 --timeout-method thread > gpurun_out/r6/s_pytest.log 2>&1
prc=$?; echo "pytest rc=$prc"; grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/r6/s_pytest.log | tail -30
[ $prc -le 1 ] || exit $prc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6/s_smoke.log 2>&1; echo "smoke rc=$?"; tail -1 gpurun_out/r6/s_smoke.log
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6/s_bench.log 2>&1; echo "bench rc=$?"; grep -o "\"value\": [0-9.]*\|\"final_loss\": [^}]*" gpurun_out/r6/s_bench.log
