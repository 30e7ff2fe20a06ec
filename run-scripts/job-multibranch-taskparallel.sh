#!/bin/bash
# Multi-branch GFM with task parallelism (reference run-scripts/job-multibranch-taskparallel.sh):
# MultiTaskModelMP — the shared encoder is data-parallel over all ranks, each decoder
# branch lives on its own rank group (branch-local gradient sync), one rank per GPU.
# Usage: run-scripts/job-multibranch-taskparallel.sh [nproc] [epochs] [workdir]
set -euo pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0 OMP_NUM_THREADS=${OMP_NUM_THREADS:-7}
NPROC=${1:-8}; EPOCHS=${2:-10}; WD=${3:-$PWD/sc25_work}
python -m torch.distributed.run --nnodes=1 --nproc-per-node "$NPROC" --master-addr 127.0.0.1 --master-port 29751 \
  examples/multibranch/train.py --task_parallel --inputfile multibranch_GFM260_SC25.json --num_epoch "$EPOCHS" \
  --workdir "$WD"
