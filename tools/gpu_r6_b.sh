set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_geometry.py > gpurun_out/t6.log 2>&1; rc=$?; tail -2 gpurun_out/t6.log; grep -E "^E  " gpurun_out/t6.log | head -10 || true
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_model_gpu.py tests/test_model_parity_gpu.py -k "SchNet or schnet" > gpurun_out/t7.log 2>&1; rc=$?; tail -2 gpurun_out/t7.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python tools/bench_configs.py qm9_schnet --steps 30 --warmup 5 > gpurun_out/b1.log 2>&1 && grep metric gpurun_out/b1.log | cut -c1-200 &&
HYDRA_RS_GRAPHS=0 timeout -k 10 300 python tools/bench_configs.py qm9_schnet --steps 30 --warmup 5 > gpurun_out/b2.log 2>&1 && grep metric gpurun_out/b2.log | cut -c1-200
