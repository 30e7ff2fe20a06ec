#!/bin/bash
# o3.Linear weight-gradient split heuristic A/B on MACE, after the o3.Linear tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in 512,128 1024,256; do
  HYDRA_IL_WG=$v timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_irreps_linear_gpu.py > gpurun_out/r6n_tests.log 2>&1 || { tail -30 gpurun_out/r6n_tests.log; exit 1; }
  echo "tests HYDRA_IL_WG=$v: $(tail -1 gpurun_out/r6n_tests.log)"
done
for v in 256,64 512,128 1024,256 256,64 512,128 1024,256; do
  echo "HYDRA_IL_WG=$v"
  HYDRA_IL_WG=$v timeout -k 10 300 python3 tools/bench_configs.py multibranch_mace --steps 40 --warmup 10 --precision fp32 2>&1 | grep metric | cut -c1-140 || exit 1
done
