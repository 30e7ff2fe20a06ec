#!/bin/bash
# Inference sweep (reference run-scripts/SC25-inference.sh): every trained model (log
# directory) evaluated on every dataset's test split; one JSON line per (model, dataset)
# with task errors and inference graphs/s, appended to inference_output_log.txt.
# One MI355X node: one rank per GPU over RCCL (torchrun), HBM-resident test loaders.
# Usage: run-scripts/SC25-inference.sh [workdir] [nproc] [models] [datasets]
#   models/datasets are comma lists; defaults match run-scripts/SC25-multibranch-*.sh outputs.
set -euo pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0 OMP_NUM_THREADS=${OMP_NUM_THREADS:-7}
WD=${1:-$PWD/sc25_work}; NPROC=${2:-8}
MODELS=${3:-GFM}; DATASETS=${4:-ANI1x,QM7-X,MPTrj,Alexandria,transition1x}
OUT=$WD/inference_output_log.txt
for m in ${MODELS//,/ }; do
  for d in ${DATASETS//,/ }; do
    [ -d "$WD/dataset/$d.bp" ] || { echo "skip $d (no store)"; continue; }
    python -m torch.distributed.run --nnodes=1 --nproc-per-node "$NPROC" --master-addr 127.0.0.1 --master-port 29731 \
      examples/multidataset/inference.py --log "$m" --datasets "$d" --workdir "$WD" | grep '^{' | tee -a "$OUT"
  done
done
