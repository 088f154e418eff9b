#!/bin/bash
# Extend the committed GEMM tuning table (engine/gemm_tuning.py): search unseen shapes for each
# workload (PDT_TUNE_GEMMS=1), then re-run read-only. New tables land in gpurun_out/tune_<model>/.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
run() { n=$1; shift; timeout -k 10 900 python -u bench.py "$@" > gpurun_out/tg_$n.log 2>&1; rc=$?
  echo "$n rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/tg_$n.log) $(grep -o 'warmup step 1/[0-9]* done at [0-9.]*' gpurun_out/tg_$n.log)"
  [ $rc -ne 0 ] && tail -5 gpurun_out/tg_$n.log; return $rc; }
for spec in "resnet50:" "vit_b16:--precision fp8"; do
  m=${spec%%:*}; extra=${spec#*:}
  rm -rf gpurun_out/tune_$m; mkdir -p gpurun_out/tune_$m
  PDT_TUNE_GEMMS=1 PDT_TUNE_GEMMS_OUT=$PWD/gpurun_out/tune_$m run ${m}_tune --model $m --steps 5 --warmup 2 $extra || exit 1
done
ls -la gpurun_out/tune_*
