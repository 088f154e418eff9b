#!/bin/bash
# Round 5 (j): PMC counters of the layer-1 weight-stationary 3x3 kernel (pinned pipeline, with and
# without its halo DMA); the damped fp32-oracle fused-vs-unfused test.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out/pmc_c3
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT"
P2="SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT"
for opt in 9 11; do
  i=0
  for pm in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $pm --output-format csv -d /tmp/pmc_${opt}_$i -o run -- python3 tools/c3_one.py $opt dgrad 3 > gpurun_out/pmc_c3/log_${opt}_$i.txt 2>&1 || { echo "pmc rc=$? opt=$opt pass=$i"; tail -5 gpurun_out/pmc_c3/log_${opt}_$i.txt; exit 1; }
    f=$(find /tmp/pmc_${opt}_$i -name "*counter_collection.csv" | head -1)
    cp "$f" gpurun_out/pmc_c3/counters_opt${opt}_pass$i.csv
  done
done
for opt in 9 11; do echo "== opt $opt"; python tools/pmc_summary.py gpurun_out/pmc_c3/counters_opt${opt}_pass1.csv/.. conv3x3wst 2>/dev/null; done
timeout -k 10 300 python -u -m pytest "tests/test_conv1x1_bwd_fused_gpu.py::test_resnet50_grads_fused_vs_unfused" -q -s --timeout 200 --timeout-method thread > gpurun_out/t_j2.log 2>&1; rc=$?
echo "oracle test rc=$rc"; grep -E "fused vs fp32|passed|failed|Error" gpurun_out/t_j2.log | head -8
exit 0
