set -o pipefail
cd $GRAFT_REPO_ROOT
run() { timeout -k 10 "$@"; rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc; }
run 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_geometry.py tests/test_multibranch_capture.py > gpurun_out/t6.log 2>&1; tail -2 gpurun_out/t6.log; grep -E "^E  |FAILED" gpurun_out/t6.log | head -10
run 300 python tools/bench_configs.py qm9_schnet --steps 30 --warmup 5 > gpurun_out/b1.log 2>&1; grep metric gpurun_out/b1.log | cut -c1-200
HYDRA_RS_GRAPHS=0 run 300 python tools/bench_configs.py qm9_schnet --steps 30 --warmup 5 > gpurun_out/b2.log 2>&1; grep metric gpurun_out/b2.log | cut -c1-200
BENCH_SINGLE_BRANCH=1 run 400 python tools/bench_configs.py multibranch_egnn multibranch_mace --steps 20 --warmup 5 > gpurun_out/b3.log 2>&1; grep metric gpurun_out/b3.log | cut -c1-260
run 400 python tools/bench_configs.py multibranch_egnn multibranch_mace --steps 20 --warmup 5 > gpurun_out/b4.log 2>&1; grep metric gpurun_out/b4.log | cut -c1-260
