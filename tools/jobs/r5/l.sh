#!/bin/bash
# Round 5 (l): row-tile 3x3 probes (41 full, 43 no DMA, 45 no MFMA) + PMC of the full and compute-only
# kernel; fp32-oracle conditioning sweep.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out/pmc_wsr
timeout -k 10 300 python -u tools/conv3x3_bench.py --opts 41,43,45 --only 64@56 > gpurun_out/c3_l.txt 2>&1; rc=$?
cat gpurun_out/c3_l.txt; [ $rc -eq 0 ] || exit $rc
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT"
P2="SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT"
for opt in 41 43; do
  i=0
  for pm in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $pm --output-format csv -d /tmp/pmcw_${opt}_$i -o run -- python3 tools/c3_one.py $opt dgrad 3 > gpurun_out/pmc_wsr/log_${opt}_$i.txt 2>&1 || { echo "pmc rc=$? opt=$opt pass=$i"; tail -5 gpurun_out/pmc_wsr/log_${opt}_$i.txt; exit 1; }
    f=$(find /tmp/pmcw_${opt}_$i -name "*counter_collection.csv" | head -1)
    cp "$f" gpurun_out/pmc_wsr/counters_opt${opt}_pass$i.csv
  done
done
echo pmc done
timeout -k 10 300 python -u tools/diag_oracle.py > gpurun_out/diag_oracle2.txt 2>&1; rc=$?
cat gpurun_out/diag_oracle2.txt | grep -v amdgpu.ids; exit $rc
