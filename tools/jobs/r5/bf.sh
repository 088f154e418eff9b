#!/bin/bash
# Round 5 (bf): TunableOp search for ResNet-50's remaining hipBLASLt GEMMs (the split-K batched 1x1 weight gradients
# of layers 2-4 and the fc: none were in the table), merged into a table copy, then the default bench with the
# committed table vs the merged one, alternating, same box.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out/tunableop /tmp/tt_old /tmp/tt_new
( export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=0 \
    PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=30 PYTORCH_TUNABLEOP_MAX_WARMUP_DURATION_MS=5 \
    PYTORCH_TUNABLEOP_FILENAME=$PWD/gpurun_out/tunableop/r50_%d.csv
  timeout -k 10 900 python -u bench.py --steps 3 --warmup 2 > gpurun_out/bf_tune.log 2>&1 ); rc=$?
echo "tune rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/bf_tune.log)"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bf_tune.log; exit $rc; }
cp tuning/tunableop_gfx950.csv /tmp/tt_old/t0.csv
python3 - <<'PY' || exit 1
tab = open("tuning/tunableop_gfx950.csv").read().splitlines()
keys = {",".join(l.split(",")[:2]) for l in tab}
new = [l.strip() for l in open("gpurun_out/tunableop/r50_0.csv") if not l.startswith("Validator") and l.strip()]
add = [l for l in new if ",".join(l.split(",")[:2]) not in keys]
open("/tmp/tt_new/t0.csv", "w").write("\n".join(tab + add) + "\n")
open("gpurun_out/tunableop/r50_added.csv", "w").write("\n".join(add) + "\n")
print("added", len(add), "entries")
PY
for v in old new old new; do
  PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=/tmp/tt_$v/t%d.csv \
    timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bf_run.log 2>&1; rc=$?
  echo "resnet50 b1024 table=$v rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/bf_run.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bf_run.log)" | tee -a gpurun_out/bf.txt
  [ $rc -eq 0 ] || { tail -20 gpurun_out/bf_run.log; exit $rc; }
done
