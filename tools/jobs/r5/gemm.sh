#!/bin/bash
# Round 5: split-K Linear GEMM — tests, then ours (split 0=auto,1,2,4) vs tuned hipBLASLt on the ViT/GPT-2 shapes.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_conv1x1_bwd_fused_gpu.py -x -v --timeout 300 \
  --timeout-method thread > gpurun_out/t_gemm.log 2>&1; rc=$?; echo "gemm+fused tests rc=$rc"; tail -5 gpurun_out/t_gemm.log
grep -E "FAILED|Error" gpurun_out/t_gemm.log | head -5; [ $rc -eq 0 ] || exit $rc
for epi in bias gelu; do
  timeout -k 10 400 python -u tools/gemm_bench.py --epi $epi --rounds 5 --splits 0,1,2,3,4,6 > gpurun_out/gemm_bench_$epi.jsonl 2>&1
  rc=$?; echo "gemm bench $epi rc=$rc"; grep shape gpurun_out/gemm_bench_$epi.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); ks=[k for k in d if k.endswith('_us')]
    print(d['shape'], d['epi'], 'auto', d['auto_split'], ' '.join(f\"{k[:-3]}={d[k]}\" for k in ks), 'best', d['best'], 'x', d['speedup'])"
  [ $rc -eq 0 ] || exit $rc
done
