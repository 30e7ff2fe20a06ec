#!/bin/bash
# A/B of the row-program interpreter's workgroup size on the md17 PAINN force config.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for t in 256 512 1024 256; do
  HYDRA_ROWPROG_THREADS=$t timeout -k 10 200 python tools/bench_configs.py md17_painn_forces --steps 30 --warmup 5 \
    > gpurun_out/ab_rp.log 2>&1 || { tail -5 gpurun_out/ab_rp.log; exit 1; }
  echo "threads $t: $(tail -1 gpurun_out/ab_rp.log | cut -c1-160)"
done
