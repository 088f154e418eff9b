#!/bin/bash
# Measured roofline of the ResNet-50 training step (1024/GPU): HBM bytes (FETCH_SIZE / WRITE_SIZE,
# one counter pass each: together they need 5 TCC counters, the block has 4) and MFMA bf16 ops per
# kernel, over the steady-state steps; tools/step_roofline.py joins them by dispatch order.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/roof
i=0
for pm in "FETCH_SIZE SQ_INSTS_VALU_MFMA_MOPS_BF16" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 400 rocprofv3 --pmc $pm --output-format csv -d /tmp/roof_$i -o run -- python3 bench.py --steps 2 --warmup 3 $BENCH_ARGS > gpurun_out/roof/log_$i.txt 2>&1 || { echo "pmc rc=$? pass=$i"; tail -5 gpurun_out/roof/log_$i.txt; exit 1; }
  f=$(find /tmp/roof_$i -name "*counter_collection.csv" | head -1)
  python3 tools/step_roofline.py --reduce "$f" gpurun_out/roof/pass$i.csv || exit 1
done
python3 tools/step_roofline.py --join gpurun_out/roof/pass1.csv gpurun_out/roof/pass2.csv > gpurun_out/roof/roofline.md
cat gpurun_out/roof/roofline.md
