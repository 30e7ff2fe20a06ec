#!/bin/bash
# multibranch MACE: native (fused TP conv + symmetric contraction) vs HYDRA_UNFUSED=tp,symcon, per-step profile
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/bench_configs.py multibranch_mace --steps 20 --warmup 5 > gpurun_out/mace_native.log 2>&1 || exit $?
echo "native   $(grep metric gpurun_out/mace_native.log | cut -c1-200)"
HYDRA_UNFUSED=symcon timeout -k 10 300 python3 -u tools/bench_configs.py multibranch_mace --steps 20 --warmup 5 > gpurun_out/mace_nosym.log 2>&1 || exit $?
echo "no-symcon $(grep metric gpurun_out/mace_nosym.log | cut -c1-200)"
HYDRA_UNFUSED=tpconv timeout -k 10 300 python3 -u tools/bench_configs.py multibranch_mace --steps 20 --warmup 5 > gpurun_out/mace_notp.log 2>&1 || exit $?
echo "no-tpconv $(grep metric gpurun_out/mace_notp.log | cut -c1-200)"
bash tools/gpu_prof_cfg.sh multibranch_mace fp32 || exit $?
