#!/bin/bash
# Round 5 (aw): TunableOp search for GPT-2-medium's fp8 GEMMs (the committed table held only its bf16 ones),
# merged into the table copy on this box, then GPT-2-medium bf16 vs fp8 on the merged table (same box).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out/tunableop
( export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=0 \
    PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=30 PYTORCH_TUNABLEOP_MAX_WARMUP_DURATION_MS=5 \
    PYTORCH_TUNABLEOP_FILENAME=$PWD/gpurun_out/tunableop/gpt2fp8_%d.csv
  timeout -k 10 600 python -u bench.py --model gpt2_medium --precision fp8 --steps 6 --warmup 3 > gpurun_out/aw_tune.log 2>&1 ); rc=$?
echo "tune rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/aw_tune.log)"; [ $rc -eq 0 ] || { tail -5 gpurun_out/aw_tune.log; exit $rc; }
python3 - <<'PY' || exit 1
import glob
new = [l for f in glob.glob("gpurun_out/tunableop/gpt2fp8_*.csv") for l in open(f) if l.startswith("ScaledGemm")]
tab = open("tuning/tunableop_gfx950.csv").read().splitlines()
keys = {",".join(l.split(",")[:2]) for l in tab}
add = [l.strip() for l in new if ",".join(l.split(",")[:2]) not in keys]
open("tuning/tunableop_gfx950.csv", "w").write("\n".join(tab + add) + "\n")
open("gpurun_out/tunableop/gpt2fp8_added.csv", "w").write("\n".join(add) + "\n")
print("added", len(add), "fp8 entries")
PY
for p in bf16 fp8 bf16 fp8; do
  timeout -k 10 400 python -u bench.py --model gpt2_medium --precision $p --steps 20 --warmup 5 > gpurun_out/aw_$p.log 2>&1; rc=$?
  echo "gpt2_medium $p rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/aw_$p.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/aw_$p.log)"; [ $rc -eq 0 ] || exit $rc
done
