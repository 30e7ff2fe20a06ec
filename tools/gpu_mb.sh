#!/bin/bash
# multibranch capture tests + config benches, then the full GPU suite and the headline bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-mb}
timeout -k 10 300 python -u -m pytest tests/test_multibranch_capture.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
grep -E "passed|failed|FAILED" gpurun_out/${TAG}_tests.log | tail -5
if [ $rc -ne 0 ]; then exit $rc; fi
for prec in fp32 bf16; do
  timeout -k 10 400 python -u tools/bench_configs.py multibranch_egnn multibranch_mace qm9_schnet --steps 20 --warmup 10 --precision $prec > gpurun_out/${TAG}_configs_$prec.log 2>&1 || exit $?
  grep metric gpurun_out/${TAG}_configs_$prec.log | cut -c1-230
done
bash tools/gpu_full_tests.sh
