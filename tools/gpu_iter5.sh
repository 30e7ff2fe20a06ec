#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "edge_linear or pna or linear" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/iter5_tests.log 2>&1
rc=$?; tail -2 gpurun_out/iter5_tests.log; [ $rc -ne 0 ] && exit $rc
for cfg in "HYDRA_EDGE_LINEAR=0" "HYDRA_EDGE_LINEAR=1" "HYDRA_EDGE_LINEAR=0" "HYDRA_EDGE_LINEAR=1"; do
  echo "== bench $cfg"; env $cfg timeout -k 10 180 python3 bench.py --steps 40 --warmup 5 2>&1 | tail -1 | cut -c1-200 || exit 1
done
bash tools/gpu_prof_bench.sh head5 > /dev/null 2>&1; grep -E "edge_linear|dispatches" gpurun_out/prof_head5_summary.txt | cut -c1-120
