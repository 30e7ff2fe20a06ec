#!/bin/bash
# Single-dataset baselines (reference run-scripts/job-baseline-singledataset{0..4}.sh and
# SC25-baseline-singledataset*.sh): train the GFM model on ONE dataset store at a time,
# all GPUs of the node as data-parallel ranks (--adios = one store, loaders shard it).
# Usage: run-scripts/job-baseline-singledataset.sh [index 0-4|all] [nproc] [epochs] [workdir]
set -euo pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0 OMP_NUM_THREADS=${OMP_NUM_THREADS:-7}
SETS=(ANI1x QM7-X MPTrj Alexandria transition1x)
IDX=${1:-all}; NPROC=${2:-8}; EPOCHS=${3:-10}; WD=${4:-$PWD/sc25_work}
run() {
  local name=$1
  python -m torch.distributed.run --nnodes=1 --nproc-per-node "$NPROC" --master-addr 127.0.0.1 --master-port 29741 \
    examples/multidataset/train.py --adios --modelname "$name" --inputfile gfm_multitasking.json \
    --num_epoch "$EPOCHS" --log "baseline_$name" --workdir "$WD" | grep '^{'
}
if [ "$IDX" = all ]; then for s in "${SETS[@]}"; do run "$s"; done; else run "${SETS[$IDX]}"; fi
