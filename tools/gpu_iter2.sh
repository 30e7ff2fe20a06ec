#!/bin/bash
# new-kernel tests first, then the perf iteration (bench A/B + tests + profile)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-iter}
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py tests/test_model_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_newtests.log 2>&1
rc=$?
tail -4 gpurun_out/${TAG}_newtests.log
if [ $rc -ne 0 ]; then exit $rc; fi
HYDRA_DEFER_WGRAD=0 timeout -k 10 200 python bench.py --steps 30 --warmup 10 > gpurun_out/${TAG}_bench_nodefer.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_bench_nodefer.log | cut -c1-200
bash tools/gpu_iter.sh $TAG
