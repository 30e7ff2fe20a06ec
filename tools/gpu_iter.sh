#!/bin/bash
# Iteration on one MI355X: kernel tests of the parts being changed, the headline
# bench, and a marked per-step kernel trace (summary + one step's timeline).
#   TESTS="tests/a.py tests/b.py" BENCH_ARGS="--precision bf16" bash tools/gpu_iter.sh [tag]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-iter}
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread $TESTS > gpurun_out/t_$TAG.log 2>&1 \
    || { tail -40 gpurun_out/t_$TAG.log; exit 1; }
  tail -2 gpurun_out/t_$TAG.log
fi
if [ -n "$PRE" ]; then eval "$PRE" || exit 1; fi
timeout -k 10 300 python bench.py --steps 30 --warmup 5 $BENCH_ARGS > gpurun_out/bench_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log
export HYDRA_PROFILE_MARK=1
OUT=gpurun_out/prof_$TAG
rm -rf $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format rocpd -d $OUT -o run -- python3 bench.py --steps 20 --warmup 5 $BENCH_ARGS > ${OUT}.log 2>&1 || { tail -20 ${OUT}.log; exit 1; }
DB=$(find $OUT -name "*.db" | head -1)
python3 tools/rocpd_summary.py $DB --between spin_kernel --steps 20 --top 40 > ${OUT}_summary.txt
python3 tools/step_timeline.py $DB --step 10 > ${OUT}_timeline.txt
head -30 ${OUT}_summary.txt
tail -4 ${OUT}_timeline.txt
rm -rf $OUT
