#!/bin/bash
# SC25-style multibranch foundation-model training on one MI355X node (reference
# run-scripts/SC25-job-weak.sh / SC25-multibranch.sh): EGNN hidden 866 x 4 layers,
# 5 branches (graph energy + node forces), batch 128 per rank, task parallel
# (MultiTaskModelMP: encoder synced over the world, each branch over its group).
# Weak scaling: per-rank work fixed, 1 -> 8 GPUs.  HYDRAGNN_MAX_NUM_BATCH caps the
# batches per epoch like the reference protocol (5 batches x 4 epochs).
set -euo pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0 HYDRAGNN_MAX_NUM_BATCH=${HYDRAGNN_MAX_NUM_BATCH:-5}
for N in 5 8; do  # task parallel needs >= 1 rank per branch (5 branches)
  python -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" --master-addr 127.0.0.1 \
    --master-port $((29700 + N)) examples/multibranch/train.py --task_parallel \
    --inputfile multibranch_GFM260_SC25.json --num_samples $((640 * N)) --num_epoch 4 \
    --workdir "logs/sc25_weak_n${N}" 2>&1 | tee "logs/sc25_weak_n${N}.log"
done
