#!/bin/bash
# BASELINE configs 2/3/5 on one GPU + rocprof summaries (DBs removed to keep gpurun_out small)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python3 tools/bench_configs.py --steps 20 --warmup 5 --precision fp32 > gpurun_out/cfg_fp32.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/bench_configs.py qm9_schnet multibranch_egnn --steps 20 --warmup 5 --precision bf16 > gpurun_out/cfg_bf16.log 2>&1 || exit $?
for c in "qm9_schnet fp32" "md17_painn_forces fp32" "multibranch_mace fp32" "multibranch_egnn bf16"; do
  bash tools/gpu_prof_cfg.sh $c > /dev/null 2>&1 || exit $?
done
rm -rf gpurun_out/prof_cfg_*_fp32 gpurun_out/prof_cfg_*_bf16
grep -h metric gpurun_out/cfg_*.log | cut -c1-160
