#!/bin/bash
# EGNN fused-path numerics, then per-step profiles: EGNN-866 captured bf16 and QM9 SchNet
# (in-forward static radius graph)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -v -s --timeout 120 --timeout-method thread tests/test_bgemm_gpu.py tests/test_egnn_wide_gpu.py tests/test_multibranch_capture.py > gpurun_out/egnn_tests.log 2>&1
rc=$?; grep -E "rel|PASS|FAIL|passed|failed|Error|error" gpurun_out/egnn_tests.log | tail -40
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_prof_cfg.sh multibranch_egnn bf16 || exit $?
bash tools/gpu_prof_cfg.sh qm9_schnet fp32 || exit $?
