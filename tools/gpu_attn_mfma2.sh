#!/bin/bash
# MFMA attention forward v2: numerics, standalone timing + per-kernel rocprof, headline bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "attention" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/attn_tests.log 2>&1
rc=$?; tail -3 gpurun_out/attn_tests.log; [ $rc -ne 0 ] && exit $rc
echo "== MFMA"; timeout -k 10 120 python3 tools/bench_attn.py 2311 8 8 2>&1 | grep splits || exit 1
rm -rf gpurun_out/prof_attn
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_attn -o run -- python3 tools/bench_attn.py 2311 8 8 > gpurun_out/prof_attn.log 2>&1 || exit 1
f=$(find gpurun_out/prof_attn -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 "$f" | head -14
echo "== bench"; timeout -k 10 180 python3 bench.py --steps 30 --warmup 5 2>&1 | tail -1 | cut -c1-220 || exit 1
