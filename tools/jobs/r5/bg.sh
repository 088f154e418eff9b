#!/bin/bash
# Round 5 (bg): 8-wave 128x64-per-wave 1x1 tile for deep-K forwards (PDT_CONV1X1_W2=1): conv tests with it on,
# per-shape probe timings off / on, then the default bench off / on / off / on.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
PDT_CONV1X1_W2=1 timeout -k 10 400 python -u -m pytest tests/test_conv1x1_ours_gpu.py tests/test_headline_shapes_gpu.py -q -x --timeout 200 --timeout-method thread > gpurun_out/t_bg.log 2>&1; rc=$?
echo "tests (W2=1) rc=$rc"; tail -1 gpurun_out/t_bg.log; grep -E "^E  |^FAILED" gpurun_out/t_bg.log | head; [ $rc -eq 0 ] || exit $rc
for w in 0 1; do
  PDT_CONV1X1_W2=$w PDT_PROBES=0,0 timeout -k 10 300 python -u tools/conv1x1_probe.py > gpurun_out/bg_probe_$w.txt 2>&1; rc=$?
  echo "== W2=$w"; grep "fwd+stats" gpurun_out/bg_probe_$w.txt; [ $rc -eq 0 ] || exit $rc
done
for w in 0 1 0 1; do
  PDT_CONV1X1_W2=$w timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bg_run.log 2>&1; rc=$?
  echo "resnet50 W2=$w rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/bg_run.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bg_run.log)" | tee -a gpurun_out/bg.txt
  [ $rc -eq 0 ] || { tail -20 gpurun_out/bg_run.log; exit $rc; }
done
