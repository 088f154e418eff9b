#!/bin/bash
# PMC counters of the 3x3 weight-gradient kernel (layer 3 shape, batch 1024): MFMA-only probe and full.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT"
P2="SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT"
for probe in 2 0; do
  i=0
  for pm in "$P1" "$P2"; do
    i=$((i+1))
    PROBE=$probe ONLY=3 timeout -s KILL 90 rocprofv3 --pmc $pm --output-format csv -d /tmp/pmc_${probe}_$i -o run -- tools/convbench/wgrad3x3_bench 1024 > gpurun_out/pmc/log_${probe}_$i.txt 2>&1 || { echo "pmc rc=$? probe=$probe pass=$i"; tail -5 gpurun_out/pmc/log_${probe}_$i.txt; exit 1; }
    f=$(find /tmp/pmc_${probe}_$i -name "*counter_collection.csv" | head -1)
    cp "$f" gpurun_out/pmc/counters_probe${probe}_pass$i.csv
  done
done
echo pmc done
