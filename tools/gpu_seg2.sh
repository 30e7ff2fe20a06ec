#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "segment or weight_prep" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/seg2_tests.log 2>&1
rc=$?
tail -2 gpurun_out/seg2_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/bench_configs.py multibranch_egnn --steps 15 --warmup 8 --precision bf16 > gpurun_out/seg2_egnn.log 2>&1 || exit $?
grep metric gpurun_out/seg2_egnn.log | cut -c1-200
timeout -k 10 200 python bench.py --steps 30 --warmup 10 > gpurun_out/seg2_bench.log 2>&1 || exit $?
tail -1 gpurun_out/seg2_bench.log | cut -c1-200
