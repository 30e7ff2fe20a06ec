#!/bin/bash
# EGNN fused-path + multibranch numerics, then per-step profiles of MACE fp32 and EGNN-866 bf16
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -v --timeout 120 --timeout-method thread tests/test_irreps_linear_gpu.py tests/test_kernels_gpu.py tests/test_bgemm_gpu.py tests/test_egnn_wide_gpu.py tests/test_multibranch_capture.py tests/test_model_parity_gpu.py -m gpu > gpurun_out/s3_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|passed|failed|Error" gpurun_out/s3_tests.log | tail -30
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_prof_cfg.sh multibranch_mace fp32 || exit $?
bash tools/gpu_prof_cfg.sh multibranch_egnn bf16 || exit $?
