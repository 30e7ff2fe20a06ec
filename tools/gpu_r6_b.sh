set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_parity_gpu.py tests/test_model_gpu.py -k "mace or MACE or segment_mean" > gpurun_out/t6.log 2>&1; tail -2 gpurun_out/t6.log; grep -E "^E  " gpurun_out/t6.log | head -10
timeout -k 10 300 python tools/bench_configs.py multibranch_mace --steps 30 --warmup 5 2>&1 | grep metric | cut -c1-200
