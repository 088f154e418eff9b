#!/bin/bash
# bench default = hipGraph-captured step at N = 1 (ResNet): graph tests, then the driver's bench command, twice
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out/r6
timeout -k 10 400 python -u -m pytest tests/test_graph_gpu.py tests/test_graph_collectives_gpu.py tests/test_determinism_gpu.py -q --timeout 240 --timeout-method thread > gpurun_out/r6/ai_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r6/ai_tests.log | tail -5
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6/ai_bench_$i.log 2>&1 || exit 3
  echo "default bench $i: $(grep -o '"value": [0-9.]*' gpurun_out/r6/ai_bench_$i.log) $(grep -o '"graph": [a-z]*' gpurun_out/r6/ai_bench_$i.log) $(grep -o '"final_loss": [0-9.]*' gpurun_out/r6/ai_bench_$i.log)"
done
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --graph 0 > gpurun_out/r6/ai_bench_eager.log 2>&1 || exit 3
echo "eager: $(grep -o '"value": [0-9.]*' gpurun_out/r6/ai_bench_eager.log) $(grep -o '"final_loss": [0-9.]*' gpurun_out/r6/ai_bench_eager.log)"
