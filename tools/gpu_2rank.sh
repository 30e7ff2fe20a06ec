#!/bin/bash
# 2 ranks on the one GPU of the box (gloo fallback: RCCL needs one GPU per rank): exercises
# the multi-rank bench path (spawn, broadcast, bucketed sync hooks, deferred wgrad flush)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --gpus 2 --steps 10 --warmup 5 > gpurun_out/bench_2rank.log 2>&1
rc=$?
tail -3 gpurun_out/bench_2rank.log | cut -c1-250
exit $rc
