#!/bin/bash
# Strong scaling of the SC25 multibranch configuration (reference run-scripts/SC25-job-strong.sh):
# global batch fixed at 640 graphs, split over the ranks (batch = 640 / N per rank).
set -euo pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0 HYDRAGNN_MAX_NUM_BATCH=${HYDRAGNN_MAX_NUM_BATCH:-5}
for N in 5 8; do
  BS=$((640 / N))
  python -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" --master-addr 127.0.0.1 \
    --master-port $((29800 + N)) examples/multibranch/train.py --task_parallel \
    --inputfile multibranch_GFM260_SC25.json --batch_size "$BS" --num_samples 3200 --num_epoch 4 \
    --workdir "logs/sc25_strong_n${N}" 2>&1 | tee "logs/sc25_strong_n${N}.log"
done
