#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_prof_bench.sh r2a || exit $?
for prec in fp32 bf16; do
  timeout -k 10 300 python tools/bench_configs.py qm9_schnet multibranch_egnn --steps 20 --warmup 10 --precision $prec > gpurun_out/configs_$prec.log 2>&1 || exit $?
  grep metric gpurun_out/configs_$prec.log | cut -c1-200
done
