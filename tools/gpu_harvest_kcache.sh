#!/bin/bash
# Populate MIOpen's compiled-kernel cache for the headline bench on a fresh box and bring it back
# under gpurun_out/ (copy it to miopen_cache/kcache afterwards: git-ignored, but it ships with the
# tree, so later fresh boxes skip the ~2 min of first-step kernel compilation).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
rm -rf gpurun_out/miopen_cache; cp -r miopen_cache gpurun_out/miopen_cache
export PDT_MIOPEN_CACHE=$PWD/gpurun_out/miopen_cache
timeout -k 10 ${TB:-240} python -u bench.py --steps 10 --warmup 3 > gpurun_out/harvest.log 2>&1; rc=$?
echo "rc=$rc"; grep -E "warmup step 1/|metric" gpurun_out/harvest.log; du -sh gpurun_out/miopen_cache/*
exit $rc
