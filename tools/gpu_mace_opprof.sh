#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
BENCH_MODE=eager BENCH_OP_PROFILE=1 BENCH_OP_SORT=count timeout -k 10 300 python3 -u tools/bench_configs.py multibranch_mace --steps 3 --warmup 3 > gpurun_out/mace_opprof.log 2>&1
