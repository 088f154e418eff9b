#!/bin/bash
# Round 5 (ap): PMC of the stem weight gradient, pooled-gradient form vs dz-reading form (batch 256).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out/pmc_stem
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT"
P2="SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT"
for m in pool dz; do
  i=0
  for pm in "$P1" "$P2"; do
    i=$((i+1))
    rm -rf /tmp/pmc_stem_${m}_$i
    timeout -s KILL 120 rocprofv3 --pmc $pm --output-format csv -d /tmp/pmc_stem_${m}_$i -o run -- python3 tools/stem_one.py $m 256 2 > gpurun_out/pmc_stem/log_${m}_$i.txt 2>&1 || { echo "pmc rc=$? $m $i"; tail -5 gpurun_out/pmc_stem/log_${m}_$i.txt; exit 1; }
    f=$(find /tmp/pmc_stem_${m}_$i -name "*counter_collection.csv" | head -1)
    cp "$f" gpurun_out/pmc_stem/${m}_$i.csv
  done
done
python3 - <<'PY'
import csv, collections
for m in ("pool", "dz"):
    tot = collections.OrderedDict()
    for i in (1, 2):
        rows = list(csv.DictReader(open(f"gpurun_out/pmc_stem/{m}_{i}.csv")))
        ids = sorted({int(r["Dispatch_Id"]) for r in rows if "stem_wgrad_kernel" in r["Kernel_Name"]})
        last = ids[-1]
        for r in rows:
            if int(r["Dispatch_Id"]) == last:
                tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    print("==", m)
    for k, v in tot.items():
        print(f"  {k:<28}{v:>18,.0f}")
    g = tot.get("GRBM_GUI_ACTIVE", 0) / 8
    if g:
        print(f"  MFMA-busy {tot['SQ_VALU_MFMA_BUSY_CYCLES'] / (1024 * g):.1%}  VALU/MFMA {tot['SQ_INSTS_VALU'] / tot['SQ_INSTS_MFMA']:.1f}"
              f"  waves {tot['SQ_WAVES']:.0f}  wait-any/wave-cycles {tot['SQ_WAIT_ANY'] / max(tot['SQ_WAVE_CYCLES'], 1):.2f}")
PY
