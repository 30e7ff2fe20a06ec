set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "tp or TP or conv" > gpurun_out/t3.log 2>&1; tail -3 gpurun_out/t3.log
timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_model_parity_gpu.py -k "MACE or mace" > gpurun_out/t4.log 2>&1; tail -2 gpurun_out/t4.log
timeout -k 10 300 python tools/bench_configs.py multibranch_mace --steps 20 --warmup 5 2>&1 | grep metric | cut -c1-200
timeout -k 10 400 bash tools/gpu_prof_cfg.sh multibranch_mace fp32 > gpurun_out/prof_mace.log 2>&1 || exit 1
grep -E "dispatches|tp_conv" gpurun_out/prof_mace.log | cut -c1-150
