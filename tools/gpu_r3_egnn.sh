#!/bin/bash
# SC25 EGNN-866 multibranch (BASELINE config 5) on the bf16 engine: eager vs captured, fp32 reference,
# then a per-step rocprof summary of the faster bf16 mode
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for cap in 0 1; do
  HYDRA_MULTIBRANCH_CAPTURE=$cap timeout -k 10 300 python3 -u tools/bench_configs.py multibranch_egnn --steps 20 --warmup 5 --precision bf16 > gpurun_out/egnn_bf16_cap$cap.log 2>&1 || exit $?
  echo "capture=$cap $(grep metric gpurun_out/egnn_bf16_cap$cap.log | cut -c1-260)"
done
timeout -k 10 300 python3 -u tools/bench_configs.py multibranch_egnn --steps 10 --warmup 3 --precision fp32 > gpurun_out/egnn_fp32.log 2>&1 || exit $?
echo "fp32 $(grep metric gpurun_out/egnn_fp32.log | cut -c1-260)"
HYDRA_MULTIBRANCH_CAPTURE=${1:-auto} bash tools/gpu_prof_cfg.sh multibranch_egnn bf16 || exit $?
