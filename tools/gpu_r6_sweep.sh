#!/bin/bash
# Round-6 configuration sweep on one GPU: every bench_configs config in fp32 and the bf16
# ones, the SC25 single-branch layout, SchNet with every map forced to bf16, and the headline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { timeout -k 10 "$@"; rc=$?; [ $rc -eq 0 ] || exit $rc; }
run 200 python3 bench.py --steps 20 --warmup 5 > gpurun_out/sw_headline.log 2>&1; tail -1 gpurun_out/sw_headline.log | cut -c1-200
run 700 python3 tools/bench_configs.py --steps 20 --warmup 5 --precision fp32 > gpurun_out/sw_fp32.log 2>&1; grep metric gpurun_out/sw_fp32.log | cut -c1-200
BENCH_SINGLE_BRANCH=1 run 400 python3 tools/bench_configs.py multibranch_egnn multibranch_mace --steps 20 --warmup 5 --precision fp32 > gpurun_out/sw_single.log 2>&1; grep metric gpurun_out/sw_single.log | cut -c1-200
run 400 python3 tools/bench_configs.py qm9_schnet multibranch_egnn --steps 20 --warmup 5 --precision bf16 > gpurun_out/sw_bf16.log 2>&1; grep metric gpurun_out/sw_bf16.log | cut -c1-200
HYDRA_BF16_MIN_MACS=0 run 300 python3 tools/bench_configs.py qm9_schnet --steps 20 --warmup 5 --precision bf16 > gpurun_out/sw_schnet_bf16_all.log 2>&1; grep metric gpurun_out/sw_schnet_bf16_all.log | cut -c1-200
run 200 python3 bench.py --steps 20 --warmup 5 > gpurun_out/sw_headline2.log 2>&1; tail -1 gpurun_out/sw_headline2.log | cut -c1-200
