#!/bin/bash
# new kernels' oracle tests + model parity, then BASELINE configs 2/3/5 benches + rocprof
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_parity_gpu.py -k "spherical or gather_mul or edge_basis or parity or gpu_matches" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/iter6_tests.log 2>&1
rc=$?; tail -3 gpurun_out/iter6_tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_cfg_prof.sh
