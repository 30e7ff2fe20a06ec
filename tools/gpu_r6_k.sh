#!/bin/bash
# force-training configs: per-step rocprof summaries at HEAD
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_prof_cfg.sh md17_pnaeq_forces fp32 || exit $?
bash tools/gpu_prof_cfg.sh md17_egnn_forces fp32 || exit $?
