#!/bin/bash
# iteration 5: single-round head-loss staging + saved activations, flat-index assembly
# element-parallel batch assembly: tests, headline (x2), profile + step timeline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_head_loss_gpu.py tests/test_fused_gpu.py tests/test_gps_fused_gpu.py tests/test_attention8_gpu.py tests/test_kernels_gpu.py > gpurun_out/r3_iter7_tests.log 2>&1
rc=$?; tail -6 gpurun_out/r3_iter7_tests.log; [ $rc -eq 0 ] || exit $rc
HYDRA_STEP_TIMING=1 timeout -k 10 240 python3 bench.py --steps 50 --warmup 10 > gpurun_out/r3_iter7_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r3_iter7_bench.log | cut -c1-400
timeout -k 10 240 python3 bench.py --steps 100 --warmup 10 > gpurun_out/r3_iter7_bench2.log 2>&1 || exit $?
tail -1 gpurun_out/r3_iter7_bench2.log | cut -c1-300
bash tools/gpu_prof_bench.sh r3_iter7 || exit $?
python3 tools/step_timeline.py gpurun_out/prof_r3_iter7/run_results.db --step 5 > gpurun_out/r3_iter7_timeline.txt 2>&1
tail -4 gpurun_out/r3_iter7_timeline.txt
