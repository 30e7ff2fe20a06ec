#!/bin/bash
# Round-6 per-step kernel tables (rocprofv3 kernel trace) of the headline and the configs
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/gpu_prof_headline_final.sh > gpurun_out/ph.log 2>&1 || exit $?
head -2 gpurun_out/prof_final_summary.txt | cut -c1-150
for c in md17_painn_forces qm9_dimenet qm9_schnet multibranch_mace; do
  bash tools/gpu_prof_cfg.sh $c fp32 > gpurun_out/pc_$c.log 2>&1 || exit $?
  head -1 gpurun_out/prof_cfg_${c}_fp32_summary.txt | cut -c1-150
done
BENCH_SINGLE_BRANCH=1 bash tools/gpu_prof_cfg.sh multibranch_egnn fp32 > gpurun_out/pc_egnn.log 2>&1 || exit $?
head -1 gpurun_out/prof_cfg_multibranch_egnn_fp32_summary.txt | cut -c1-150
