set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_branch_mlp_gpu.py > gpurun_out/t3.log 2>&1; tail -30 gpurun_out/t3.log | grep -E "Error|error|assert|Mismatch|passed|failed" | head -20
timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_model_parity_gpu.py -k "MACE or mace" > gpurun_out/t4.log 2>&1; tail -2 gpurun_out/t4.log
timeout -k 10 300 python tools/bench_configs.py multibranch_mace --steps 20 --warmup 5 2>&1 | grep metric | cut -c1-200
HYDRA_BRANCH_MLP=0 timeout -k 10 300 python tools/bench_configs.py multibranch_mace --steps 20 --warmup 5 2>&1 | grep metric | cut -c1-200
