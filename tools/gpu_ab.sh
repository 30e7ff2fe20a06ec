#!/bin/bash
# headline bench A/B over env settings (each its own bounded run), then the GPU model tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-ab}
i=0
for envs in "" "HYDRA_GPS_FORK=0" "HYDRA_BRANCH_STREAMS=0"; do
  i=$((i+1))
  env $envs timeout -k 10 200 python bench.py --steps 30 --warmup 10 > gpurun_out/${TAG}_bench$i.log 2>&1 || { echo "bench $i ($envs) failed"; tail -30 gpurun_out/${TAG}_bench$i.log; exit 1; }
  echo "[$envs] $(tail -1 gpurun_out/${TAG}_bench$i.log | cut -c1-150)"
done
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py tests/test_model_parity_gpu.py tests/test_fused_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_tests.log
exit $rc
