#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fused_gpu.py -k "egnn or gat or cg or mf" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/egnn_tests.log 2>&1
rc=$?
tail -3 gpurun_out/egnn_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for prec in fp32 bf16; do
  timeout -k 10 300 python -u tools/bench_configs.py multibranch_egnn --steps 15 --warmup 8 --precision $prec > gpurun_out/egnn_$prec.log 2>&1 || exit $?
  grep metric gpurun_out/egnn_$prec.log | cut -c1-200
done
