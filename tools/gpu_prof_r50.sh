#!/bin/bash
# ResNet-50 bench + steady-state kernel profile; keeps the raw trace for neighbour analysis.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 $BENCH_ARGS > gpurun_out/bench_r50.log 2>&1; rc=$?
grep -E "warmup step 1/|metric" gpurun_out/bench_r50.log; [ $rc -eq 0 ] || exit $rc
rm -rf /tmp/p_r50; mkdir -p /tmp/p_r50
timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --output-format csv -d /tmp/p_r50 -o run -- python3 bench.py --steps 5 --warmup 3 $BENCH_ARGS > gpurun_out/prof_r50.log 2>&1
rc=$?; echo "prof rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/prof_r50.log)"; [ $rc -eq 0 ] || exit $rc
python tools/prof_window.py /tmp/p_r50 gpurun_out/steady_r50${TAG} timed 5 > /dev/null
head -3 gpurun_out/steady_r50${TAG}.md
mkdir -p gpurun_out/trace_r50
cp $(find /tmp/p_r50 -name "*kernel_trace.csv") gpurun_out/trace_r50/kernel_trace.csv
cp $(find /tmp/p_r50 -name "*marker_api_trace.csv") gpurun_out/trace_r50/marker_api_trace.csv
ls -la gpurun_out/trace_r50
