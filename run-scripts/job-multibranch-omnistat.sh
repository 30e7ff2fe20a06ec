#!/bin/bash
# Multi-branch training with node telemetry (reference run-scripts/*-omnistat.sh, which
# wraps the job in Omnistat GPU/energy sampling).  Here: rocm-smi samples GPU use,
# power and memory every second into $WD/telemetry.csv while the job runs, and the
# energy (integrated board power) is summarised at the end.
# Usage: run-scripts/job-multibranch-omnistat.sh [nproc] [epochs] [workdir]
set -euo pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0 OMP_NUM_THREADS=${OMP_NUM_THREADS:-7}
NPROC=${1:-8}; EPOCHS=${2:-10}; WD=${3:-$PWD/sc25_work}
mkdir -p "$WD"
TEL=$WD/telemetry.csv
( while true; do
    echo "# $(date +%s.%N)"; rocm-smi --showuse --showpower --showmemuse --csv 2>/dev/null || true
    sleep 1
  done ) > "$TEL" &
SAMPLER=$!
trap 'kill $SAMPLER 2>/dev/null || true' EXIT
python -m torch.distributed.run --nnodes=1 --nproc-per-node "$NPROC" --master-addr 127.0.0.1 --master-port 29761 \
  examples/multibranch/train.py --inputfile multibranch_GFM260_SC25.json --num_epoch "$EPOCHS" --workdir "$WD"
kill $SAMPLER 2>/dev/null || true
python - "$TEL" <<'PY'
import sys, re
t, watts = [], []
cur = None
for line in open(sys.argv[1]):
    if line.startswith("# "):
        cur = float(line[2:]); continue
    m = re.findall(r"(\d+\.\d+)", line) if "card" in line.lower() else []
    if m and cur is not None:
        t.append(cur); watts.append(float(m[0]))
if len(t) > 1:
    import numpy as np
    print(f"samples {len(t)}  mean power {np.mean(watts):.1f} W  energy ~{np.trapz(watts, t) / 3600:.3f} Wh")
PY
