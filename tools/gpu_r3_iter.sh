#!/bin/bash
# iteration: attention8 numerics + microbench, fused encoder tests, headline bench (+ PNA A/B), profile
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention8_gpu.py tests/test_gps_fused_gpu.py > gpurun_out/r3_iter_tests.log 2>&1
rc=$?; tail -6 gpurun_out/r3_iter_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 tools/bench_attn8.py > gpurun_out/r3_iter_attn.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r3_iter_attn.log
for v in 0 1; do
  HYDRA_PNA_WAVE=$v HYDRA_STEP_TIMING=1 timeout -k 10 240 python3 bench.py --steps 50 --warmup 10 > gpurun_out/r3_iter_bench_pna$v.log 2>&1 || exit $?
  echo "PNA_WAVE=$v: $(tail -1 gpurun_out/r3_iter_bench_pna$v.log | cut -c1-160)"
done
bash tools/gpu_prof_bench.sh r3_iter || exit $?
