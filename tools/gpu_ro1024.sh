#!/bin/bash
# Read-only ResNet-50 run at 1024 images/GPU with the harvested caches; Python stacks every 45 s
# show where the first (warm-up) step spends its time.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
rm -rf gpurun_out/miopen_cache; cp -r miopen_cache gpurun_out/miopen_cache
export PDT_MIOPEN_CACHE=$PWD/gpurun_out/miopen_cache
PDT_STACK_DUMP=45 timeout -k 10 ${T:-540} python -u bench.py --batch-size ${B:-1024} --steps 20 --warmup 5 > gpurun_out/ro_b${B:-1024}.log 2>&1; rc=$?
echo "rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/ro_b${B:-1024}.log) $(grep -o 'warmup step 1/[0-9]* done at [0-9.]*' gpurun_out/ro_b${B:-1024}.log)"
exit $rc
