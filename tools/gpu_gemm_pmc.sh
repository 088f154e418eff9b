#!/bin/bash
# PMC counters of the Linear GEMM (tools/convbench/gemm_bench_g4) on one shape, one pass per counter set.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
shape=${1:-gpt2_fc1}
mkdir -p gpurun_out/pmc_gemm
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT"
P2="SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT"
P3="TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr TD_BUSY_avr"
i=0
for pm in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $pm --output-format csv -d /tmp/pmcg_$i -o run -- tools/convbench/gemm_bench_g4 $shape > gpurun_out/pmc_gemm/log_$i.txt 2>&1 || { echo "pmc rc=$? pass=$i"; tail -5 gpurun_out/pmc_gemm/log_$i.txt; exit 1; }
  f=$(find /tmp/pmcg_$i -name "*counter_collection.csv" | head -1)
  cp "$f" gpurun_out/pmc_gemm/counters_pass$i.csv
done
echo pmc done
