#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_profile_gate_gpu.py -q -x --timeout 200 --timeout-method thread -k "batchnorm or stem or bn_ or resnet" > gpurun_out/stem_tests.log 2>&1; rc=$?
tail -2 gpurun_out/stem_tests.log; [ $rc -eq 0 ] || exit $rc
rm -rf /tmp/p_s; mkdir -p /tmp/p_s
timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --output-format csv -d /tmp/p_s -o run -- python3 bench.py --steps 5 --warmup 3 > gpurun_out/prof_s.log 2>&1 || exit 1
grep -o '"value": [0-9.]*' gpurun_out/prof_s.log
python tools/prof_window.py /tmp/p_s gpurun_out/steady_stem timed 5 > /dev/null
grep -E "pool|Window" gpurun_out/steady_stem.md | cut -c1-160
