set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_branch_mlp_gpu.py tests/test_mace_radial_gpu.py > gpurun_out/t3.log 2>&1; tail -3 gpurun_out/t3.log
timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_model_parity_gpu.py tests/test_model_gpu.py -k "MACE or mace" > gpurun_out/t4.log 2>&1; tail -2 gpurun_out/t4.log
timeout -k 10 300 python tools/bench_configs.py multibranch_mace --steps 30 --warmup 5 2>&1 | grep metric | cut -c1-200
