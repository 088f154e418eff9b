#!/bin/bash
# Round 5 (ab): ResNet-50 1024/GPU with every round-5 change: bench x2, step window + categories, PMC roofline.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_ab$i.log 2>&1; rc=$?
  echo "bench $i rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/bench_ab$i.log)"; [ $rc -eq 0 ] || exit $rc
done
rm -rf /tmp/p_r50; mkdir -p /tmp/p_r50
timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --output-format csv -d /tmp/p_r50 -o run -- python3 bench.py --steps 5 --warmup 3 > gpurun_out/prof_r50.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python tools/prof_window.py /tmp/p_r50 gpurun_out/steady_resnet50_b1024 timed 5 > /dev/null && head -1 gpurun_out/steady_resnet50_b1024.md
python tools/prof_categories.py gpurun_out/steady_resnet50_b1024_kernels.csv > gpurun_out/steady_resnet50_b1024_categories.md 2>/dev/null; cat gpurun_out/steady_resnet50_b1024_categories.md
bash tools/gpu_step_roofline.sh
