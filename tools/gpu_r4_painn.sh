#!/bin/bash
# Round-4 GPU step: the F=32 fused-encoder fault diagnostic (op-level sync), then the
# native PAINN force kernels and a md17 PAINN force bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
HYDRA_DEBUG_SYNC=1 AMD_SERIALIZE_KERNEL=3 timeout -k 10 200 python -u -m pytest -x -q --timeout 120 \
  --timeout-method thread "tests/test_gps_fused_gpu.py::test_fused_encoder_matches_module_path[32-0.25]" \
  > gpurun_out/diag32.log 2>&1
rc=$?
grep -v "^frame" gpurun_out/diag32.log | tail -30
if [ $rc -ne 0 ]; then exit 1; fi
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_painn_force_gpu.py \
  > gpurun_out/painn_gpu.log 2>&1 || { grep -v "^frame" gpurun_out/painn_gpu.log | tail -60; exit 1; }
tail -8 gpurun_out/painn_gpu.log
timeout -k 10 300 python -u tools/bench_configs.py md17_painn_forces --steps 20 --warmup 5 > gpurun_out/bench_painn.log 2>&1 \
  || { tail -30 gpurun_out/bench_painn.log; exit 1; }
tail -3 gpurun_out/bench_painn.log
