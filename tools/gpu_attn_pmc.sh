#!/bin/bash
# Flash-attention kernel timings (tools/attn_bench.py) + two PMC passes over the same run.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/pmc_attn
timeout -k 10 120 python -u tools/attn_bench.py > gpurun_out/attn_bench.txt 2>&1 || exit $?
cat gpurun_out/attn_bench.txt
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT"
P2="SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for pm in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pm --output-format csv -d /tmp/pmca_$i -o run -- python3 tools/attn_bench.py > gpurun_out/pmc_attn/log_$i.txt 2>&1 || { echo "pmc rc=$? pass=$i"; tail -5 gpurun_out/pmc_attn/log_$i.txt; exit 1; }
  f=$(find /tmp/pmca_$i -name "*counter_collection.csv" | head -1)
  cp "$f" gpurun_out/pmc_attn/counters_pass$i.csv
done
echo pmc done
