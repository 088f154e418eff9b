#!/bin/bash
# PMC counters of the 3x3 conv kernel at one ResNet-50 layer (ONLY=1..4), one pass per run.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp NOREF=1 ONLY=${ONLY:-3}
mkdir -p gpurun_out/pmc
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_LDS_ADDR_CONFLICT SQ_INST_LEVEL_LDS"
P3="TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VMEM SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_VMEM_TA_CMD_FIFO_FULL GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $P --kernel-trace --output-format csv -d gpurun_out/pmc/p$i -o p$i -- ./tools/convbench/conv3x3_bench 3 > gpurun_out/pmc/p$i.log 2>&1 || exit $?
done
