#!/bin/bash
# L2 (TCC) hit/miss counters per kernel of the headline step: do the CSR neighbour gathers
# (pna / segment / edge kernels) hit in L2?  One counter pass, kernel trace only.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/pmc_l2
rm -rf $OUT
timeout -s KILL 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $OUT -o run -- python3 bench.py --steps 5 --warmup 3 > ${OUT}.log 2>&1 || exit $?

python3 tools/pmc_summary.py $OUT > gpurun_out/pmc_l2_summary.txt 2>&1 || true
head -40 gpurun_out/pmc_l2_summary.txt
rm -rf $OUT
