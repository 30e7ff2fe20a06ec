set -o pipefail
cd $GRAFT_REPO_ROOT
run() { timeout -k 10 "$@"; rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc; }
run 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_irreps_linear_gpu.py tests/test_multibranch_capture.py tests/test_mace_radial_gpu.py tests/test_branch_mlp_gpu.py > gpurun_out/t9.log 2>&1; tail -2 gpurun_out/t9.log; grep -E "^E  |FAILED" gpurun_out/t9.log | head -10
run 300 python tools/bench_configs.py multibranch_mace --steps 30 --warmup 5 > gpurun_out/b6.log 2>&1; grep metric gpurun_out/b6.log | cut -c1-200
BENCH_SINGLE_BRANCH=1 run 300 python tools/bench_configs.py multibranch_mace --steps 30 --warmup 5 > gpurun_out/b7.log 2>&1; grep metric gpurun_out/b7.log | cut -c1-200
