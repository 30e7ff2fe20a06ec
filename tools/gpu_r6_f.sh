set -o pipefail
cd $GRAFT_REPO_ROOT
run() { timeout -k 10 "$@"; rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc; }
run 500 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_fused_gpu.py tests/test_egnn_wide_gpu.py tests/test_mace_radial_gpu.py tests/test_multibranch_capture.py > gpurun_out/t9.log 2>&1; tail -2 gpurun_out/t9.log; grep -E "^E  |FAILED" gpurun_out/t9.log | head -10
BENCH_SINGLE_BRANCH=1 run 400 python tools/bench_configs.py multibranch_egnn --steps 20 --warmup 5 > gpurun_out/b6.log 2>&1; grep metric gpurun_out/b6.log | cut -c1-200
run 400 python tools/bench_configs.py multibranch_egnn --steps 20 --warmup 5 > gpurun_out/b7.log 2>&1; grep metric gpurun_out/b7.log | cut -c1-200
