set -o pipefail
cd $GRAFT_REPO_ROOT
run() { timeout -k 10 "$@"; rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc; }
run 500 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_forces.py tests/test_painn_force_gpu.py > gpurun_out/t9.log 2>&1; tail -2 gpurun_out/t9.log; grep -E "^E  |FAILED" gpurun_out/t9.log | head -10
for v in 1 0; do
HYDRA_COMPOSITE_SPLITK=$v run 400 python tools/bench_configs.py md17_egnn_forces md17_pnaeq_forces --steps 20 --warmup 5 > gpurun_out/b6.log 2>&1; echo "splitk=$v"; grep metric gpurun_out/b6.log | cut -c1-150
done
