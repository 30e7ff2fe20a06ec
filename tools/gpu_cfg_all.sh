#!/bin/bash
# BASELINE configs 2/3/5 on one GPU (fp32 + bf16 where it applies) + rocprof summaries
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python3 tools/bench_configs.py --steps 20 --warmup 5 --precision fp32 > gpurun_out/cfg_fp32.log 2>&1 || exit $?
grep metric gpurun_out/cfg_fp32.log | cut -c1-220
timeout -k 10 300 python3 tools/bench_configs.py qm9_schnet multibranch_egnn --steps 20 --warmup 5 --precision bf16 > gpurun_out/cfg_bf16.log 2>&1 || exit $?
grep metric gpurun_out/cfg_bf16.log | cut -c1-220
bash tools/gpu_prof_cfg.sh qm9_schnet bf16 > /dev/null 2>&1 || exit $?
bash tools/gpu_prof_cfg.sh md17_painn_forces fp32 > /dev/null 2>&1 || exit $?
bash tools/gpu_prof_cfg.sh multibranch_mace fp32 > /dev/null 2>&1 || exit $?
ls gpurun_out/*_summary.txt
