#!/bin/bash
# MACE fused linear chain: numerics, MACE GPU tests, then the config bench and rocprof summary
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_irreps_linear_gpu.py tests/test_model_parity_gpu.py tests/test_kernels_gpu.py tests/test_mace_radial_gpu.py tests/test_multibranch_capture.py > gpurun_out/r6h_tests.log 2>&1 || { tail -30 gpurun_out/r6h_tests.log; exit 1; }
tail -2 gpurun_out/r6h_tests.log
bash tools/gpu_prof_cfg.sh multibranch_mace fp32 || exit $?
timeout -k 10 300 python3 tools/bench_configs.py multibranch_mace --steps 30 --warmup 10 --precision fp32 2>&1 | grep metric | cut -c1-200
