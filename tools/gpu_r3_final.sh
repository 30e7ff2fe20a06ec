#!/bin/bash
# round-end evidence in one call: numerics of the recently changed paths, then the
# headline bench + per-step profile, EGNN-866, BASELINE config sweep + profiles, L2 counters
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -v --timeout 120 --timeout-method thread tests/test_irreps_linear_gpu.py tests/test_kernels_gpu.py tests/test_multibranch_capture.py tests/test_model_parity_gpu.py -m gpu > gpurun_out/final_tests.log 2>&1
rc=$?; grep -E "FAIL|passed|failed|Error" gpurun_out/final_tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_r3_perf.sh || exit $?
