#!/bin/bash
# Round 5 (o): row-tile 3x3 with the BN backward reduction (opt bit 7): tests, A/B, bench; fp32 diag.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_headline_shapes_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_o1.log 2>&1; rc=$?
echo "headline tests rc=$rc"; tail -2 gpurun_out/t_o1.log; grep -E "^E  |Error" gpurun_out/t_o1.log | head -10; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/conv3x3_bench.py --opts 41,169 --only 64@56 > gpurun_out/c3_o.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/c3_o.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_o.log 2>&1; rc=$?
echo "bench rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/bench_o.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/diag_oracle.py > gpurun_out/diag_oracle4.txt 2>&1; rc=$?
grep -v "amdgpu.ids\|Warning\|detach\|return float" gpurun_out/diag_oracle4.txt | tail -20; exit $rc
