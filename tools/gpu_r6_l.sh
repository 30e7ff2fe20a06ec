#!/bin/bash
# force configs after routing composite Linear+ReLU through the split-K linear; tests first
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_forces.py tests/test_fused_gpu.py > gpurun_out/r6l_tests.log 2>&1 || { tail -30 gpurun_out/r6l_tests.log; exit 1; }
tail -1 gpurun_out/r6l_tests.log
for c in md17_egnn_forces md17_pnaeq_forces; do
  timeout -k 10 300 python3 tools/bench_configs.py $c --steps 30 --warmup 10 --precision fp32 2>&1 | grep metric | cut -c1-140 || exit 1
done
bash tools/gpu_prof_cfg.sh md17_egnn_forces fp32 || exit $?
