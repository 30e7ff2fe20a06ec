#!/bin/bash
# o3.Linear forward rows-per-workgroup A/B on MACE, after the o3.Linear tests at each setting
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in 8; do
  HYDRA_IL_ROWS=$v timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_irreps_linear_gpu.py > gpurun_out/r6p_tests.log 2>&1 || { tail -30 gpurun_out/r6p_tests.log; exit 1; }
  echo "tests HYDRA_IL_ROWS=$v: $(tail -1 gpurun_out/r6p_tests.log)"
done
for v in 4 8 4 8; do
  echo "HYDRA_IL_ROWS=$v"
  HYDRA_IL_ROWS=$v timeout -k 10 300 python3 tools/bench_configs.py multibranch_mace --steps 40 --warmup 10 --precision fp32 2>&1 | grep metric | cut -c1-140 || exit 1
done
