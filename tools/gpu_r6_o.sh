#!/bin/bash
# ReLU-epilogue A/B on the GPS module-path configs (their FFN's Linear+ReLU)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in 1 0 1 0; do
  echo "HYDRA_LINEAR_RELU_EPI=$v"
  HYDRA_LINEAR_RELU_EPI=$v timeout -k 10 300 python3 tools/bench_configs.py qm9_schnet_gps oc20_gps_h128 --steps 30 --warmup 10 --precision fp32 2>&1 | grep metric | cut -c1-120 || exit 1
done
