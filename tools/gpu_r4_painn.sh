#!/bin/bash
# Round-4 GPU step: native PAINN force kernels (tests), md17 PAINN force bench + per-step profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_painn_force_gpu.py \
  > gpurun_out/painn_gpu.log 2>&1 || { grep -v "^frame" gpurun_out/painn_gpu.log | tail -60; exit 1; }
tail -3 gpurun_out/painn_gpu.log
bash tools/gpu_prof_cfg.sh md17_painn_forces fp32
