#!/bin/bash
# Round 5 (be): same-box A/B of the 11 GPT-2-medium fp8 TunableOp entries: the committed table vs the same table
# without them, GPT-2-medium fp8, graphed, alternating.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out /tmp/tt_with /tmp/tt_without
cp tuning/tunableop_gfx950.csv /tmp/tt_with/t0.csv
grep -v "^ScaledGemm.*_8192_" tuning/tunableop_gfx950.csv > /tmp/tt_without/t0.csv
echo "entries: with $(grep -c ScaledGemm /tmp/tt_with/t0.csv), without $(grep -c ScaledGemm /tmp/tt_without/t0.csv)"
for v in with without with without; do
  PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=/tmp/tt_$v/t%d.csv \
    timeout -k 10 400 python -u bench.py --model gpt2_medium --precision fp8 --graph 1 --steps 20 --warmup 5 > gpurun_out/be_run.log 2>&1; rc=$?
  echo "gpt2 fp8 graph table=$v rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/be_run.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/be_run.log)" | tee -a gpurun_out/be.txt
  [ $rc -eq 0 ] || { tail -20 gpurun_out/be_run.log; exit $rc; }
done
