#!/bin/bash
# Round 5 (g): new headline-shape tests + 3x3 tests, bench x2, profile window, coverage gate.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_headline_shapes_gpu.py tests/test_conv1x1_ours_gpu.py tests/test_conv_s2_gpu.py \
  tests/test_conv_gpu.py tests/test_p2p_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_g.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/t_g.log; grep -E "^FAILED|^E  " gpurun_out/t_g.log | head -8; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_g$i.log 2>&1; rc=$?
  echo "bench $i rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/bench_g$i.log)"; [ $rc -eq 0 ] || exit $rc
done
rm -rf /tmp/p_r50; mkdir -p /tmp/p_r50
timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --output-format csv -d /tmp/p_r50 -o run -- python3 bench.py --steps 5 --warmup 3 > gpurun_out/prof_r50.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python tools/prof_window.py /tmp/p_r50 gpurun_out/steady_resnet50_b1024 timed 5 > /dev/null && head -1 gpurun_out/steady_resnet50_b1024.md
python tools/prof_categories.py gpurun_out/steady_resnet50_b1024_kernels.csv > gpurun_out/steady_resnet50_b1024_categories.md 2>/dev/null; cat gpurun_out/steady_resnet50_b1024_categories.md
cp gpurun_out/steady_resnet50_b1024_kernels.csv /tmp/step_kernels.csv
sed -i 's#profiles/r5/steady_resnet50_b1024_kernels.csv#/tmp/step_kernels.csv#' tools/gpu_coverage.sh
bash tools/gpu_coverage.sh
