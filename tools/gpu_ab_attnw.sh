#!/bin/bash
# A/B of the v2 attention kernels' waves per workgroup (HYDRA_ATTN_SPLITS=-W) inside the headline step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in 0 -4 -6 0 -4; do
  HYDRA_ATTN_SPLITS=$v timeout -k 10 200 python bench.py --steps 40 --warmup 5 > gpurun_out/ab_w.log 2>&1 || { tail -5 gpurun_out/ab_w.log; exit 1; }
  echo "splits $v: $(tail -1 gpurun_out/ab_w.log | cut -c1-150)"
done
