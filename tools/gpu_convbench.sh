cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
python -c "from pytorch_distributed_training_example_amd.engine.miopen_cache import use_repo_miopen_cache as u; print(u())"
export MIOPEN_USER_DB_PATH=$PWD/miopen_cache/db MIOPEN_CUSTOM_CACHE_DIR=$PWD/miopen_cache/kcache
timeout -k 10 500 python -u tools/conv_bench.py > gpurun_out/conv_bench.log 2>&1; rc=$?
cat gpurun_out/conv_bench.log; exit $rc
