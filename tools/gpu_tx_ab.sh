#!/bin/bash
# Transformer A/B: bench.py (driver command shape) for each extra-flag set given as arguments,
# per model in $MODELS (default: gpt2_medium vit_b16). One line per run in gpurun_out/tx_ab.txt.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
for m in ${MODELS:-gpt2_medium vit_b16}; do
  for flags in "$@"; do
    timeout -k 10 400 python3 bench.py --model $m $flags --gpus 1 --steps 20 --warmup 5 > gpurun_out/tx_ab_run.log 2>&1
    rc=$?
    echo "$m [$flags] rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/tx_ab_run.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/tx_ab_run.log)" | tee -a gpurun_out/tx_ab.txt
    [ $rc -eq 0 ] || { tail -20 gpurun_out/tx_ab_run.log; exit $rc; }
  done
done
