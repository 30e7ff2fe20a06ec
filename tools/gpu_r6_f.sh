set -o pipefail
cd $GRAFT_REPO_ROOT
run() { timeout -k 10 "$@"; rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc; }
run 600 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_fused_gpu.py tests/test_egnn_wide_gpu.py tests/test_forces.py tests/test_multibranch_capture.py tests/test_model_gpu.py tests/test_model_parity_gpu.py -k "EGNN or egnn or orce or multibranch" > gpurun_out/t9.log 2>&1; tail -2 gpurun_out/t9.log; grep -E "^E  |FAILED" gpurun_out/t9.log | head -10
for v in 1 0; do
HYDRA_LINEAR_RELU_EPI=$v BENCH_SINGLE_BRANCH=1 run 400 python tools/bench_configs.py multibranch_egnn --steps 20 --warmup 5 > gpurun_out/b6.log 2>&1; echo "epi=$v $(grep metric gpurun_out/b6.log | cut -c1-150)"
done
