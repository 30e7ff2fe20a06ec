#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
for envs in "HYDRA_SEG_VEC2=1" "HYDRA_SEG_VEC2=0"; do
  env $envs timeout -k 10 300 python -u tools/bench_configs.py multibranch_egnn --steps 40 --warmup 20 --precision bf16 > gpurun_out/egab.log 2>&1 || exit $?
  echo "[$envs] $(grep metric gpurun_out/egab.log | cut -c60-140)"
done
done
