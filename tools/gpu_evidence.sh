#!/bin/bash
# Round evidence in one call: LeNet (reference workload) eager + graphed at 128/rank; ResNet-50 at the
# reference's 128/rank (host overhead, eager, graphed, rocprofv3 window of the graphed run); then the
# transformer configs (tools/gpu_tx_prof.sh). Every GPU step under its own time limit, chained.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
val() { grep -o '"value": [0-9.]*, "unit": "[a-z/]*", "n_gpus": 1, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*' "$1"; }
for g in 0 1; do
  timeout -k 10 300 python -u bench.py --model lenet --batch-size 128 --steps 200 --warmup 20 --graph $g > gpurun_out/lenet128_g$g.log 2>&1
  rc=$?; echo "lenet graph=$g rc=$rc $(val gpurun_out/lenet128_g$g.log)"; [ $rc -eq 0 ] || exit $rc
done
bash tools/gpu_strong128.sh || exit 1
rm -rf /tmp/p_s128; mkdir -p /tmp/p_s128
timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --output-format csv -d /tmp/p_s128 -o run -- python3 bench.py --global-batch 128 --graph 1 --steps 10 --warmup 5 > gpurun_out/prof_s128.log 2>&1
rc=$?; echo "prof s128 rc=$rc"; [ $rc -eq 0 ] || exit $rc
python tools/prof_window.py /tmp/p_s128 gpurun_out/steady_resnet50_b128_graph timed 10 > /dev/null && head -1 gpurun_out/steady_resnet50_b128_graph.md
bash tools/gpu_tx_prof.sh
