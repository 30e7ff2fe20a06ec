set -o pipefail
cd $GRAFT_REPO_ROOT
run() { timeout -k 10 "$@"; rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc; }
run 500 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_multibranch_capture.py tests/test_model_gpu.py tests/test_model_parity_gpu.py -k "MACE or mace or multibranch" > gpurun_out/t9.log 2>&1; tail -2 gpurun_out/t9.log; grep -E "^E  |FAILED" gpurun_out/t9.log | head -10
run 300 python tools/bench_configs.py multibranch_mace --steps 40 --warmup 5 > gpurun_out/b6.log 2>&1; grep metric gpurun_out/b6.log | cut -c1-150
bash tools/gpu_prof_cfg.sh multibranch_mace fp32 > gpurun_out/pm.log 2>&1; head -1 gpurun_out/prof_cfg_multibranch_mace_fp32_summary.txt
