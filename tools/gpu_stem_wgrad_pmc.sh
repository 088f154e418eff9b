#!/bin/bash
# PMC counters of the stem weight-gradient kernel (tools/convbench/stem_bench_p0 WGRAD=1).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp WGRAD=1
mkdir -p gpurun_out/pmc_stemwg
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS"
timeout -s KILL 90 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d gpurun_out/pmc_stemwg/p1 -o p1 -- ./tools/convbench/stem_bench_p0 > gpurun_out/pmc_stemwg/p1.log 2>&1
