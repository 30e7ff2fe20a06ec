set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_schnet_filter_gpu.py > gpurun_out/t3.log 2>&1; tail -3 gpurun_out/t3.log
timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_forces.py tests/test_model_parity_gpu.py -k "dime or Dime" > gpurun_out/t4.log 2>&1; tail -2 gpurun_out/t4.log
timeout -k 10 300 python tools/bench_configs.py qm9_dimenet --steps 30 --warmup 5 2>&1 | grep metric | cut -c1-200
HYDRA_UNFUSED=resmlp timeout -k 10 300 python tools/bench_configs.py qm9_dimenet --steps 30 --warmup 5 2>&1 | grep metric | cut -c1-200
