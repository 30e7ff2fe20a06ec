#!/bin/bash
# bf16 engine numerics + microbench, then the round-3 full check (suite, bench, profile)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -v -s --timeout 120 --timeout-method thread tests/test_bgemm_gpu.py tests/test_egnn_wide_gpu.py > gpurun_out/bg_tests.log 2>&1
rc=$?; grep -E "rel|col|PASS|FAIL|passed|failed" gpurun_out/bg_tests.log | tail -150
timeout -k 10 200 python3 -u tools/bench_bgemm.py > gpurun_out/bg_bench.log 2>&1 || exit $?
cat gpurun_out/bg_bench.log
[ "$1" = "full" ] && bash tools/gpu_r3_full.sh r3_full
exit 0
