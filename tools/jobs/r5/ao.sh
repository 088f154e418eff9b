#!/bin/bash
# Round 5 (ao): GELU on packed fp32 pairs: tests, producer bandwidth, ViT / GPT-2 bf16 vs fp8.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_fp8_gpu.py tests/test_kernels_gpu.py tests/test_gemm_gpu.py tests/test_models_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/t_ao1.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 gpurun_out/t_ao1.log; grep -E "^E  |^FAILED" gpurun_out/t_ao1.log | head; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python3 tools/fp8_cast_bench.py > gpurun_out/fp8_cast_bench_ao.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/fp8_cast_bench_ao.txt
run() {
  local tag=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/ao_$tag.log 2>&1; local rc=$?
  echo "$tag rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/ao_$tag.log)"; return $rc
}
for i in 1 2; do
  run vit_bf16_$i python3 bench.py --model vit_b16 --steps 20 --warmup 5 || exit 1
  run vit_fp8_$i python3 bench.py --model vit_b16 --precision fp8 --steps 20 --warmup 5 || exit 1
done
run gpt_bf16 python3 bench.py --model gpt2_medium --steps 10 --warmup 3 || exit 1
run gpt_fp8 python3 bench.py --model gpt2_medium --precision fp8 --steps 10 --warmup 3 || exit 1
