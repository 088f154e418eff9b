#!/bin/bash
# What the round-end driver runs, in its order: GPU test tier (-x), smoke, bench (N=1 default args).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/drv_pytest.log 2>&1
prc=$?; echo "pytest rc=$prc"; tail -3 gpurun_out/drv_pytest.log
[ $prc -le 1 ] || exit $prc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/drv_smoke.log 2>&1
src=$?; echo "smoke rc=$src"; tail -1 gpurun_out/drv_smoke.log; [ $src -eq 0 ] || exit $src
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/drv_bench.log 2>&1
brc=$?; echo "bench rc=$brc"; grep -E "metric|warmup step 1/" gpurun_out/drv_bench.log
[ $brc -eq 0 ] || exit $brc
exit $prc
