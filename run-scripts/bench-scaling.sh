#!/bin/bash
# Headline benchmark scaling sweep on one MI355X node: OC20 PNAPlus+GPS training
# graphs/s at 1, 2, 4, 8 GPUs (weak scaling, 32 graphs per GPU per step; one rank per
# GPU over RCCL/xGMI).  Each run prints one JSON line; efficiency = value(N) / (N * value(1)).
# Usage: run-scripts/bench-scaling.sh [steps] [warmup]
set -euo pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
STEPS=${1:-50}; WARMUP=${2:-10}
mkdir -p logs/bench
for N in 1 2 4 8; do
  if [ "$N" -eq 1 ]; then
    python bench.py --gpus 1 --steps "$STEPS" --warmup "$WARMUP" | tee "logs/bench/scale_n${N}.json"
  else
    python -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" --master-addr 127.0.0.1 \
      --master-port $((29500 + N)) bench.py --gpus "$N" --steps "$STEPS" --warmup "$WARMUP" \
      | tee "logs/bench/scale_n${N}.json"
  fi
done
python - <<'PY'
import json
v = {n: json.loads(open(f"logs/bench/scale_n{n}.json").read().strip().splitlines()[-1])["value"] for n in (1, 2, 4, 8)}
for n, x in v.items():
    print(f"N={n}: {x:.1f} graphs/s, efficiency {x / (n * v[1]):.3f}")
PY
