#!/bin/bash
# attention: numerics, standalone timing MFMA on/off, per-kernel rocprof, headline bench on/off
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "attention" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/attn_tests.log 2>&1
rc=$?; tail -3 gpurun_out/attn_tests.log; [ $rc -ne 0 ] && exit $rc
for cfg in "HYDRA_ATTN_MFMA=0" "HYDRA_ATTN_MFMA=1"; do
  echo "== $cfg"; env $cfg timeout -k 10 120 python3 tools/bench_attn.py 2311 8 8 2>&1 | grep splits || exit 1
done
rm -rf gpurun_out/prof_attn
timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/prof_attn -o run --output-format rocpd -- python3 tools/bench_attn.py 2311 8 8 > gpurun_out/prof_attn.log 2>&1 || exit 1
for cfg in "HYDRA_ATTN_MFMA=0" "HYDRA_ATTN_MFMA=1"; do
  echo "== bench $cfg"; env $cfg timeout -k 10 180 python3 bench.py --steps 30 --warmup 5 2>&1 | tail -1 | cut -c1-200 || exit 1
done
