#!/bin/bash
# GPU tests + steady-state (timed-window) kernel profiles for the three north-star models (ours).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
[ -n "$SKIP_TESTS" ] || timeout -k 10 600 python -m pytest tests/test_models_gpu.py -q -x > gpurun_out/pytest_models.log 2>&1
rc=$?; echo "pytest models rc=$rc"; tail -25 gpurun_out/pytest_models.log | grep -E "passed|failed|Error|assert|FAIL" | head
if [ $rc -gt 1 ]; then exit $rc; fi
for m in ${MODELS:-resnet50 vit_b16 gpt2_medium}; do
  rm -rf /tmp/p_$m; mkdir -p /tmp/p_$m
  timeout -k 10 500 rocprofv3 --kernel-trace --marker-trace --output-format csv -d /tmp/p_$m -o run -- python3 bench.py --model $m --steps 5 --warmup 3 $BENCH_ARGS > gpurun_out/prof_$m.log 2>&1
  rc=$?; echo "prof $m rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/prof_$m.log)"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/prof_$m.log; exit $rc; fi
  python tools/prof_window.py /tmp/p_$m gpurun_out/steady_$m${TAG} timed 5 > /dev/null
  head -3 gpurun_out/steady_$m${TAG}.md
done
