#!/bin/bash
# Round-4 measurement of the other BASELINE configurations on one MI355X (tools/bench_configs.py),
# one process per config and precision, each under its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/r4_configs.log
: > $OUT
for spec in "qm9_schnet fp32" "md17_painn_forces fp32" "multibranch_egnn fp32" "multibranch_egnn bf16" \
            "multibranch_mace fp32" "qm9_schnet bf16"; do
  set -- $spec
  timeout -k 10 300 python tools/bench_configs.py $1 --precision $2 --steps 20 --warmup 5 > gpurun_out/cfg_$1_$2.log 2>&1 \
    || { echo "$1 $2 FAILED rc=$?" >> $OUT; tail -5 gpurun_out/cfg_$1_$2.log >> $OUT; exit 1; }
  tail -1 gpurun_out/cfg_$1_$2.log | cut -c1-400 >> $OUT
done
cat $OUT
