#!/bin/bash
# One GPU call: full GPU suite, EGNN-866 bench + per-step profile, BASELINE config sweep + profiles,
# headline bench + per-step profile.  Each step has its own time limit; a crash stops the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/all_tests.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/all_tests.log | tail -15
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/gpu_r3_egnn.sh || exit $?
bash tools/gpu_r3_cfgs.sh || exit $?
HYDRA_STEP_TIMING=1 timeout -k 10 240 python3 bench.py --steps 50 --warmup 10 > gpurun_out/headline_bench.log 2>&1 || exit $?
tail -1 gpurun_out/headline_bench.log | cut -c1-600
bash tools/gpu_prof_bench.sh r3_headline || exit $?
bash tools/gpu_pmc_l2.sh || exit $?
exit $rc
