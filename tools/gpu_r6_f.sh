set -o pipefail
cd $GRAFT_REPO_ROOT
run() { timeout -k 10 "$@"; rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc; }
run 500 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_dimenet_sbf_gpu.py tests/test_forces.py tests/test_model_gpu.py tests/test_model_parity_gpu.py -k "imenet or IME or lowrank" > gpurun_out/t9.log 2>&1; tail -2 gpurun_out/t9.log; grep -E "^E  |FAILED" gpurun_out/t9.log | head -10
for v in 1 0; do
HYDRA_DIMENET_LOWRANK=$v run 300 python tools/bench_configs.py qm9_dimenet --steps 30 --warmup 5 > gpurun_out/b6.log 2>&1; echo "lowrank=$v $(grep metric gpurun_out/b6.log | cut -c1-150)"
done
