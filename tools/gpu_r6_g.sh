#!/bin/bash
# MACE: where the remaining small kernels come from, and the per-step rocprof summary
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OP_STACKS_MODE=dispatch OP_STACKS_SHAPES=1 timeout -k 10 300 python3 tools/op_stacks.py multibranch_mace > gpurun_out/stacks_mace7.txt 2>&1 || exit $?
bash tools/gpu_prof_cfg.sh multibranch_mace fp32
