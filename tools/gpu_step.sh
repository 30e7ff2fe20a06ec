#!/bin/bash
# Kernel tests + bench on the GPU box. Usage: tools/gpu_step.sh <tag> [pytest targets...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
tag=$1; shift
tests=${@:-tests/test_gemm_gpu.py}
timeout -k 10 600 python -u -m pytest $tests -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${tag}_tests.log 2>&1
rc=$?
tail -15 gpurun_out/${tag}_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 180 python bench.py --steps 20 --warmup 5 > gpurun_out/${tag}_bench.log 2>&1 || exit $?
tail -1 gpurun_out/${tag}_bench.log | cut -c1-400
exit $rc
