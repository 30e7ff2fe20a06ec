#!/bin/bash
# round-3 baseline: headline bench with host phase timing, then a marked rocprof trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
HYDRA_STEP_TIMING=1 timeout -k 10 240 python3 bench.py --steps 50 --warmup 10 > gpurun_out/r3_base_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r3_base_bench.log | cut -c1-900
timeout -k 10 240 python3 tools/bench_attn.py > gpurun_out/r3_base_attn.log 2>&1 || exit $?
tail -20 gpurun_out/r3_base_attn.log
bash tools/gpu_prof_bench.sh r3_base
