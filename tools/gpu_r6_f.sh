set -o pipefail
cd $GRAFT_REPO_ROOT
run() { timeout -k 10 "$@"; rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc; }
run 500 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_forces.py > gpurun_out/t9.log 2>&1; tail -2 gpurun_out/t9.log; grep -E "^E  |FAILED" gpurun_out/t9.log | head -10
