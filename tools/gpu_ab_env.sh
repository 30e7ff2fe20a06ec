#!/bin/bash
# A/B of environment knobs, interleaved over ROUNDS rounds (default: the headline bench):
#   VARIANTS="A= B=HYDRA_ATTN_SPLITS=-4" ROUNDS=2 bash tools/gpu_ab_env.sh
#   VARIANTS="t256=HYDRA_ROWPROG_THREADS=256 t512=HYDRA_ROWPROG_THREADS=512" \
#     BENCH_CMD="python tools/bench_configs.py md17_painn_forces --steps 30 --warmup 5" bash tools/gpu_ab_env.sh
# (multiple variables in one variant: comma-separated, A=X=1,Y=2)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
CMD=${BENCH_CMD:-"python bench.py --steps 40 --warmup 5"}
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in $VARIANTS; do
    name=${v%%=*}; envs=${v#*=}
    out=$(env $(echo $envs | tr ',' ' ') timeout -k 10 200 $CMD 2>/dev/null | grep metric | tail -1) || exit 1
    echo "$name round $r: $(echo $out | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["unit"], d["ms_per_step"], "ms/step")')"
  done
done
