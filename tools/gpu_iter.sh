#!/bin/bash
# perf iteration: bench with and without branch streams, GPU model/parity tests, rocprof of the headline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-iter}
timeout -k 10 200 python bench.py --steps 30 --warmup 10 > gpurun_out/${TAG}_bench.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-260
HYDRA_BRANCH_STREAMS=0 timeout -k 10 200 python bench.py --steps 30 --warmup 10 > gpurun_out/${TAG}_bench_1s.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_bench_1s.log | cut -c1-260
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py tests/test_model_parity_gpu.py tests/test_fused_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/gpu_prof_bench.sh $TAG || exit $?
exit $rc
