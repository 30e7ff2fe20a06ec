#!/bin/bash
# Round-4 GPU step: wgrad shape sweep + the F=32 fused-encoder test (descriptor-range fix),
# the native PAINN force kernels, and a md17 PAINN force bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_wgrad_shapes_gpu.py \
  "tests/test_gps_fused_gpu.py::test_fused_encoder_matches_module_path" > gpurun_out/fix32.log 2>&1 \
  || { grep -v "^frame" gpurun_out/fix32.log | tail -30; exit 1; }
tail -2 gpurun_out/fix32.log
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_painn_force_gpu.py \
  > gpurun_out/painn_gpu.log 2>&1 || { grep -v "^frame" gpurun_out/painn_gpu.log | tail -60; exit 1; }
tail -8 gpurun_out/painn_gpu.log
timeout -k 10 300 python -u tools/bench_configs.py md17_painn_forces --steps 20 --warmup 5 > gpurun_out/bench_painn.log 2>&1 \
  || { tail -30 gpurun_out/bench_painn.log; exit 1; }
tail -3 gpurun_out/bench_painn.log
