#!/bin/bash
# Round 5 (ba): re-run TunableOp's search for ViT-B/16's fp8 GEMMs with a longer per-solution budget (200 ms vs
# 20 ms) into a fresh table; keep an entry where it beats the committed one; ViT fp8 vs bf16 graphed on the result.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out/tunableop
( export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=0 \
    PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=200 PYTORCH_TUNABLEOP_MAX_WARMUP_DURATION_MS=20 \
    PYTORCH_TUNABLEOP_FILENAME=$PWD/gpurun_out/tunableop/vitfp8_%d.csv
  timeout -k 10 900 python -u bench.py --model vit_b16 --precision fp8 --steps 3 --warmup 2 > gpurun_out/ba_tune.log 2>&1 ); rc=$?
echo "tune rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/ba_tune.log; exit $rc; }
python3 - <<'PY' || exit 1
import glob
new = {}
for f in glob.glob("gpurun_out/tunableop/vitfp8_*.csv"):
    for l in open(f):
        if l.startswith("ScaledGemm"):
            p = l.strip().split(","); new[",".join(p[:2])] = (p[2], float(p[3]), l.strip())
tab = open("tuning/tunableop_gfx950.csv").read().splitlines()
out, changed = [], []
for l in tab:
    p = l.split(",")
    k = ",".join(p[:2])
    if k in new and len(p) >= 4 and new[k][1] < 0.97 * float(p[3]):
        changed.append(f"{k}: {p[2]} {float(p[3])*1e3:.1f} us -> {new[k][0]} {new[k][1]*1e3:.1f} us")
        out.append(new[k][2])
    else:
        out.append(l)
open("tuning/tunableop_gfx950.csv", "w").write("\n".join(out) + "\n")
open("gpurun_out/tunableop/vitfp8_changed.txt", "w").write("\n".join(changed) + "\n")
print(len(changed), "entries improved"); print("\n".join(changed))
import shutil; shutil.copy("tuning/tunableop_gfx950.csv", "gpurun_out/tunableop/merged_table.csv")
PY
for p in bf16 fp8 bf16 fp8; do
  timeout -k 10 400 python -u bench.py --model vit_b16 --precision $p --graph 1 --steps 20 --warmup 5 > gpurun_out/ba_run.log 2>&1; rc=$?
  echo "vit_b16 $p graph rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/ba_run.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ba_run.log)"
  [ $rc -eq 0 ] || { tail -20 gpurun_out/ba_run.log; exit $rc; }
done
