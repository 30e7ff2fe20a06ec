#!/bin/bash
# Captured force-step tests + md17 force bench, then the full GPU suite.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_forces.py tests/test_examples.py -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/forces_tests.log 2>&1
rc=$?
grep -E "passed|failed|FAILED" gpurun_out/forces_tests.log | tail -12
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/bench_configs.py md17_painn_forces --steps 30 --warmup 10 > gpurun_out/md17_bench.log 2>&1 || exit $?
tail -2 gpurun_out/md17_bench.log | cut -c1-400
exec_rc=0
bash tools/gpu_full_tests.sh || exec_rc=$?
exit $(( rc > exec_rc ? rc : exec_rc ))
