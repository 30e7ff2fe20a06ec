#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/op_stacks.py ${1:-multibranch_mace} > gpurun_out/op_stacks_${1:-multibranch_mace}.log 2>&1
