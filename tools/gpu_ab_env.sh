#!/bin/bash
# A/B of environment knobs on the headline bench, interleaved over ROUNDS rounds:
#   VARIANTS="A= B=HYDRA_CAPTURE_PRIORITY=-1" ROUNDS=2 bash tools/gpu_ab_env.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in $VARIANTS; do
    name=${v%%=*}; envs=${v#*=}
    out=$(env $(echo $envs | tr ',' ' ') timeout -k 10 200 python bench.py --steps 40 --warmup 5 2>/dev/null | grep metric) || exit 1
    echo "$name round $r: $(echo $out | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], "ms/step", d["config"]["host_phases_ms"])')"
  done
done
