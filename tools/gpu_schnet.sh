#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-sch}
timeout -k 10 300 python -u -m pytest tests/test_multibranch_capture.py tests/test_graphs.py -m gpu -k "capture or SchNet" -x -q --timeout 250 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for prec in fp32 bf16; do
  timeout -k 10 300 python -u tools/bench_configs.py qm9_schnet --steps 30 --warmup 10 --precision $prec > gpurun_out/${TAG}_qm9_$prec.log 2>&1 || exit $?
  grep metric gpurun_out/${TAG}_qm9_$prec.log | cut -c1-260
done
