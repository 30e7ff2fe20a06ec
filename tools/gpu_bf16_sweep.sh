#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for thr in 1073741824 16777216 0; do
  HYDRA_BF16_LIBRARY_MIN=$thr timeout -k 10 400 python -u tools/bench_configs.py multibranch_egnn qm9_schnet --steps 15 --warmup 8 --precision bf16 > gpurun_out/bf16sw.log 2>&1 || { tail -5 gpurun_out/bf16sw.log; exit 1; }
  grep metric gpurun_out/bf16sw.log | python3 -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print('thr=$thr', d['config'], d['value'], d['ms_per_step'])"
done
