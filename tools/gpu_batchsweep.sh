cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
rm -rf gpurun_out/miopen_cache; cp -r miopen_cache gpurun_out/miopen_cache
export PDT_MIOPEN_CACHE=$PWD/gpurun_out/miopen_cache
for b in 256 384 512; do
timeout -k 10 400 python -u bench.py --steps 15 --warmup 5 --batch-size $b > gpurun_out/b_bs$b.log 2>&1 || exit 1
echo "bs $b $(grep -o '"value": [0-9.]*' gpurun_out/b_bs$b.log) $(grep -o 'warmup step 1/5 done at [0-9.]*' gpurun_out/b_bs$b.log)"
done
