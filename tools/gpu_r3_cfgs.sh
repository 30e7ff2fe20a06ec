#!/bin/bash
# BASELINE configs 2/3/5 on one MI355X at HEAD + per-step (marked) rocprof summaries
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u tools/bench_configs.py --steps 20 --warmup 5 --precision fp32 > gpurun_out/cfg_fp32.log 2>&1 || exit $?
grep metric gpurun_out/cfg_fp32.log | cut -c1-260
timeout -k 10 400 python3 -u tools/bench_configs.py qm9_schnet multibranch_egnn multibranch_mace --steps 20 --warmup 5 --precision bf16 > gpurun_out/cfg_bf16.log 2>&1 || exit $?
grep metric gpurun_out/cfg_bf16.log | cut -c1-260
for c in "multibranch_mace fp32" "md17_painn_forces fp32" "qm9_schnet bf16"; do
  bash tools/gpu_prof_cfg.sh $c > /dev/null 2>&1 || exit $?
done
ls gpurun_out/*_summary.txt
