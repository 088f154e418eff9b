#!/bin/bash
# final evidence on the final defaults: per-call windows (b1024, b128 graphed), PMC step roofline, then the driver's
# order (GPU tier, smoke, bench)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out/r6
bash tools/gpu_prof_calls.sh || exit 1
bash tools/gpu_step_roofline.sh > gpurun_out/r6/final_roof.log 2>&1 || { echo roofline failed; exit 1; }
tail -14 gpurun_out/r6/final_roof.log | head -3
bash tools/gpu_strong128.sh && bash tools/jobs/r6/s.sh
