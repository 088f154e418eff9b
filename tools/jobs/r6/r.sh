#!/bin/bash
# same-box A/B of knobs on the current defaults: baseline / PDT_DS_ALG=256 / PDT_STRIDED_BSTATS=0
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out/r6
i=0
for cfg in base PDT_DS_ALG=256 PDT_STRIDED_BSTATS=0 base PDT_DS_ALG=256 PDT_STRIDED_BSTATS=0; do
  i=$((i+1))
  if [ "$cfg" = base ]; then envs=""; else envs="$cfg"; fi
  env $envs timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r6/r_bench_$i.log 2>&1 || exit 3
  echo "$cfg $(grep -o '"value": [0-9.]*' gpurun_out/r6/r_bench_$i.log)"
done
