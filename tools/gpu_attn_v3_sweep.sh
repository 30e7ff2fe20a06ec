#!/bin/bash
# v3 attention sweep: HYDRA_ATTN8_V3_R = group caps (fwd, dQ, dK/dV), HYDRA_ATTN8_V3_PERCU
set -e
mkdir -p gpurun_out
out=gpurun_out/r5_attn8_v3_sweep.log
: > $out
for cfg in ${CFGS:-1,1,1:1 1,1,1:2 2,1,1:1 2,2,2:1 3,2,2:1 4,3,3:1}; do
  r=${cfg%%:*}; pc=${cfg##*:}
  echo "== R $r per-CU $pc" >> $out
  HYDRA_ATTN8_V3_R=$r HYDRA_ATTN8_V3_PERCU=$pc timeout -k 10 120 python -u tools/bench_attn8.py 2560 2311 2>&1 | grep -E "v3 auto|W=8" >> $out
done
