#!/bin/bash
# Full GPU suite (one process) then the 1-GPU bench; stops at the first crash/timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gputests_full.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/gputests_full.log | tail -2
grep FAILED gpurun_out/gputests_full.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 180 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_full.log 2>&1 || exit $?
tail -1 gpurun_out/bench_full.log | cut -c1-300
exit $rc
