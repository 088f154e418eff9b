#!/bin/bash
# Round 5 (v): stem pooled-dz diagnostic, full GPU tier, bench x2, step profile.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/diag_stem_pool.py > gpurun_out/diag_stem_pool.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/diag_stem_pool.txt | tail -16; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/t_v_all.log 2>&1; rc=$?
echo "gpu tier rc=$rc"; tail -3 gpurun_out/t_v_all.log; grep -E "^FAILED" gpurun_out/t_v_all.log | head -10
[ $rc -le 1 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_v$i.log 2>&1; rc=$?
  echo "bench $i rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/bench_v$i.log)"; [ $rc -eq 0 ] || exit $rc
done
rm -rf /tmp/p_r50; mkdir -p /tmp/p_r50
timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --output-format csv -d /tmp/p_r50 -o run -- python3 bench.py --steps 5 --warmup 3 > gpurun_out/prof_r50.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python tools/prof_window.py /tmp/p_r50 gpurun_out/steady_resnet50_b1024 timed 5 > /dev/null && head -1 gpurun_out/steady_resnet50_b1024.md
python tools/prof_categories.py gpurun_out/steady_resnet50_b1024_kernels.csv > gpurun_out/steady_resnet50_b1024_categories.md 2>/dev/null; cat gpurun_out/steady_resnet50_b1024_categories.md
