#!/bin/bash
# v3 attention kernels: numerics tests, standalone timing (v1/sk vs v3 QPL 1/2), headline bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -k "attn or attention or gps or GPS" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/attn_tests.log 2>&1
rc=$?; tail -3 gpurun_out/attn_tests.log; [ $rc -ne 0 ] && exit $rc
for cfg in "HYDRA_ATTN_V3=0" "HYDRA_ATTN_QPL=1" "HYDRA_ATTN_QPL=2"; do
  echo "== $cfg"; env $cfg timeout -k 10 120 python3 tools/bench_attn.py 2311 8 8 2>&1 | grep splits || exit 1
done
for cfg in "HYDRA_ATTN_V3=0" "HYDRA_ATTN_QPL=1" "HYDRA_ATTN_QPL=2"; do
  echo "== bench $cfg"; env $cfg timeout -k 10 180 python3 bench.py --steps 30 --warmup 5 2>&1 | tail -1 | cut -c1-200 || exit 1
done
