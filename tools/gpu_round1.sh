#!/bin/bash
# First GPU pass: kernel numerics, smoke, bench (ours graph/eager, stock torch DDP).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_kernels_gpu.py -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -5 gpurun_out/smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 10 --warmup 5 --graph 0 > gpurun_out/bench_ours_eager.log 2>&1
rc=$?; echo "bench eager rc=$rc"; tail -3 gpurun_out/bench_ours_eager.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 10 --warmup 5 --impl torch_ddp > gpurun_out/bench_torch.log 2>&1
rc=$?; echo "bench torch rc=$rc"; tail -3 gpurun_out/bench_torch.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 10 --warmup 5 --graph 1 > gpurun_out/bench_ours_graph.log 2>&1
rc=$?; echo "bench graph rc=$rc"; tail -3 gpurun_out/bench_ours_graph.log
exit $rc
