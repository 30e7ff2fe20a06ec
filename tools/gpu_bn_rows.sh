#!/bin/bash
# A/B of the fused BatchNorm slab height (HY_BN_ROWS = 2 / 4 / 8 rows per thread):
# numerics tests per variant, then the headline bench interleaved 3x per variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in bn2 bn8; do
  HYDRA_NATIVE_LIB=$PWD/hydragnn_amd/_C_$v.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "batchnorm" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/bnrows_$v.log 2>&1
  rc=$?; echo "$v: $(tail -1 gpurun_out/bnrows_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
for i in 1 2 3; do
  for v in C C_bn2 C_bn8; do
    echo -n "$v "
    HYDRA_NATIVE_LIB=$PWD/hydragnn_amd/_$v.so timeout -k 10 180 python3 bench.py --steps 50 --warmup 10 2>&1 | tail -1 | cut -c1-190 || exit 1
  done
done
