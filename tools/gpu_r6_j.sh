#!/bin/bash
# o3.Linear forward unroll A/B (MACE), after its numerics tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_irreps_linear_gpu.py > gpurun_out/r6j_tests.log 2>&1 || { tail -30 gpurun_out/r6j_tests.log; exit 1; }
tail -1 gpurun_out/r6j_tests.log
for u in 4 16 8 4 16; do
  echo "unroll=$u"
  HYDRA_IL_UNROLL=$u timeout -k 10 300 python3 tools/bench_configs.py multibranch_mace --steps 40 --warmup 10 --precision fp32 2>&1 | grep metric | cut -c1-140 || exit 1
done
