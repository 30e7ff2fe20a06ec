#!/bin/bash
# EGNN-866 bench + profile, BASELINE config sweep + per-step profiles, headline bench + profile,
# L2 counter pass.  Each step has its own time limit; a crash stops the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
HYDRA_STEP_TIMING=1 timeout -k 10 240 python3 bench.py --steps 50 --warmup 10 > gpurun_out/headline_bench.log 2>&1 || exit $?
tail -1 gpurun_out/headline_bench.log | cut -c1-700
bash tools/gpu_prof_bench.sh r3_headline || exit $?
bash tools/gpu_r3_egnn.sh || exit $?
bash tools/gpu_r3_cfgs.sh || exit $?
bash tools/gpu_pmc_l2.sh || exit $?
