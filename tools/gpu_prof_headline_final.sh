#!/bin/bash
# Headline per-step kernel table + one step's multi-queue timeline (rocprofv3 kernel trace)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HYDRA_PROFILE_MARK=1
OUT=gpurun_out/prof_final
rm -rf $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format rocpd -d $OUT -o run -- python3 bench.py --steps 20 --warmup 5 > ${OUT}.log 2>&1 || exit $?
DB=$(find $OUT -name "*.db" | head -1)
python3 tools/rocpd_summary.py $DB --between spin_kernel --steps 20 --top 40 > ${OUT}_summary.txt
python3 tools/step_timeline.py $DB --step 10 > ${OUT}_timeline.txt
tail -1 ${OUT}.log | cut -c1-200
head -3 ${OUT}_summary.txt
tail -6 ${OUT}_timeline.txt
rm -rf $OUT
