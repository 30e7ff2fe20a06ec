#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_parity_gpu.py -k "pna or PNA" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/iter7_tests.log 2>&1
rc=$?; tail -2 gpurun_out/iter7_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do timeout -k 10 180 python3 bench.py --steps 50 --warmup 10 2>&1 | tail -1 | cut -c1-190 || exit 1; done
bash tools/gpu_prof_bench.sh i7 > /dev/null 2>&1 && head -1 gpurun_out/prof_i7_summary.txt && grep -c Cat gpurun_out/prof_i7_summary.txt
rm -rf gpurun_out/prof_i7
