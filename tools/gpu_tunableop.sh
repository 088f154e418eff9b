#!/bin/bash
# PyTorch TunableOp (hipBLASLt/rocBLAS solution search per GEMM shape): tune on GPT-2 / ViT / ResNet,
# then re-run reading the tuned CSV only. Results land in gpurun_out/tunableop/.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/tunableop
run() { n=$1; shift; timeout -k 10 600 python -u bench.py "$@" > gpurun_out/tu_$n.log 2>&1; rc=$?
  echo "$n rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/tu_$n.log) $(grep -o 'warmup step 1/[0-9]* done at [0-9.]*' gpurun_out/tu_$n.log)"
  [ $rc -ne 0 ] && tail -5 gpurun_out/tu_$n.log; return $rc; }
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_VERBOSE=0
export PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=20 PYTORCH_TUNABLEOP_MAX_WARMUP_DURATION_MS=5
for m in gpt2_medium vit_b16; do
  export PYTORCH_TUNABLEOP_FILENAME=$PWD/gpurun_out/tunableop/${m}%d.csv
  PYTORCH_TUNABLEOP_TUNING=1 run ${m}_tune --model $m --steps 10 --warmup 3 || exit 1
  PYTORCH_TUNABLEOP_TUNING=0 run ${m}_tuned --model $m --steps 10 --warmup 3 || exit 1
  PYTORCH_TUNABLEOP_ENABLED=0 run ${m}_plain --model $m --steps 10 --warmup 3 || exit 1
done
ls -la gpurun_out/tunableop
