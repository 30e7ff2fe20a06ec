#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
for envs in "HYDRA_ATTN_SPLITS=0" "HYDRA_ATTN_SPLITS=3" "HYDRA_ATTN_SPLITS=4" "HYDRA_ATTN_LDS=1 HYDRA_ATTN_SPLITS=3" "HYDRA_ATTN_LDS=1"; do
  env $envs timeout -k 10 120 python bench.py --steps 50 --warmup 10 > gpurun_out/sweep.log 2>&1 || { echo "[$envs] failed"; tail -5 gpurun_out/sweep.log; exit 1; }
  echo "[$envs] $(tail -1 gpurun_out/sweep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
done
