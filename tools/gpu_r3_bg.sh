#!/bin/bash
# bf16 engine + wide EGNN + DimeNet SBF numerics, engine microbench, EGNN-866 config bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -v -s --timeout 120 --timeout-method thread tests/test_bgemm_gpu.py tests/test_egnn_wide_gpu.py tests/test_dimenet_sbf_gpu.py tests/test_kernels_gpu.py tests/test_geometry.py tests/test_multibranch_capture.py > gpurun_out/bg_tests.log 2>&1
rc=$?; grep -E "rel|PASS|FAIL|passed|failed|Error|error" gpurun_out/bg_tests.log | tail -80
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python3 -u tools/bench_bgemm.py > gpurun_out/bg_bench.log 2>&1 || exit $?
cat gpurun_out/bg_bench.log
# (test failures reported above; the benches still run)
[ "$1" = "egnn" ] && bash tools/gpu_r3_egnn.sh
exit 0
