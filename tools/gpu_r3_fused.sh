#!/bin/bash
# fused GPS encoder: GPU numerics tests, then headline bench fused vs module path
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gps_fused_gpu.py > gpurun_out/r3_fused_tests.log 2>&1
rc=$?
tail -25 gpurun_out/r3_fused_tests.log
[ $rc -eq 0 ] || exit $rc
HYDRA_STEP_TIMING=1 timeout -k 10 240 python3 bench.py --steps 50 --warmup 10 > gpurun_out/r3_fused_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r3_fused_bench.log | cut -c1-700
bash tools/gpu_prof_bench.sh r3_fused
