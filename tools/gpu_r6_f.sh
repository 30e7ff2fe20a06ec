set -o pipefail
cd $GRAFT_REPO_ROOT
run() { timeout -k 10 "$@"; rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc; }
run 500 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_forces.py tests/test_pna_agg_gpu.py tests/test_model_parity_gpu.py -k "minmax or orce or pna or PNA or Eq" > gpurun_out/t9.log 2>&1; tail -2 gpurun_out/t9.log; grep -E "^E  |FAILED" gpurun_out/t9.log | head -10
run 400 python tools/bench_configs.py md17_pnaeq_forces md17_egnn_forces md17_painn_forces --steps 30 --warmup 5 > gpurun_out/b6.log 2>&1; grep metric gpurun_out/b6.log | cut -c1-140
