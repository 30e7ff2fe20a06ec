#!/bin/bash
# Round 3 check at HEAD: full GPU suite (one process), headline bench x2 (with host phases), rocprof per-step summary.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r3_full}
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/${TAG}_tests.log | tail -2
grep FAILED gpurun_out/${TAG}_tests.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
HYDRA_STEP_TIMING=1 timeout -k 10 240 python3 bench.py --steps 50 --warmup 10 > gpurun_out/${TAG}_bench.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-600
timeout -k 10 240 python3 bench.py > gpurun_out/${TAG}_bench_default.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_bench_default.log | cut -c1-300
bash tools/gpu_prof_bench.sh ${TAG} || exit $?
exit $rc
