#!/bin/bash
# iteration 2: wgrad narrow path + pooled encoder + PNA wave default: tests, headline, profile
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_gpu.py tests/test_gps_fused_gpu.py tests/test_kernels_gpu.py tests/test_rccl_capture_gpu.py -k "wgrad or fused or pna or rccl" > gpurun_out/r3_iter2_tests.log 2>&1
rc=$?; tail -6 gpurun_out/r3_iter2_tests.log; [ $rc -eq 0 ] || exit $rc
HYDRA_STEP_TIMING=1 timeout -k 10 240 python3 bench.py --steps 50 --warmup 10 > gpurun_out/r3_iter2_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r3_iter2_bench.log | cut -c1-700
bash tools/gpu_prof_bench.sh r3_iter2 || exit $?
