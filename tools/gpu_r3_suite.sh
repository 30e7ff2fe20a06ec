#!/bin/bash
# full GPU test suite (one process, per-test time limits)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/all_tests.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/all_tests.log | tail -15
exit $rc
