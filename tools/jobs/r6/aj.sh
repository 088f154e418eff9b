#!/bin/bash
# graph-mode NaN at 1024/GPU: whole-model fwd+bwd, eager vs replayed graph, at 1024 and 128
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out/r6
for b in 1024 128; do
  timeout -k 10 400 python3 -u tools/diag_graph_model.py --batch-size $b > gpurun_out/r6/aj_$b.log 2>&1
  rc=$?; echo "b=$b rc=$rc"; grep -v "^\[bench\]" gpurun_out/r6/aj_$b.log | tail -30; [ $rc -eq 0 ] || exit $rc
done
