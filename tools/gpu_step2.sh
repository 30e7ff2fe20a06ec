#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_geometry.py tests/test_resume.py "tests/test_graphs.py::test_train_gpu_lengths[PNA]" -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/step2_tests.log 2>&1
rc=$?
tail -5 gpurun_out/step2_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for prec in fp32 bf16; do
  timeout -k 10 300 python tools/bench_configs.py qm9_schnet multibranch_egnn --steps 10 --warmup 3 --precision $prec > gpurun_out/configs_$prec.log 2>&1 || exit $?
  grep metric gpurun_out/configs_$prec.log | cut -c1-260
done
exit $rc
