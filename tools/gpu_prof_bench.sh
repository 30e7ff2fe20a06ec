#!/bin/bash
# rocprofv3 kernel trace of the headline bench (timed steps bracketed by sleep markers)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HYDRA_PROFILE_MARK=1
OUT=gpurun_out/prof_${1:-bench}
rm -rf $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format rocpd -d $OUT -o run -- python3 bench.py --steps 20 --warmup 5 ${@:2} > ${OUT}.log 2>&1 || exit $?
DB=$(find $OUT -name "*.db" | head -1)
python3 tools/rocpd_summary.py $DB --between spin_kernel --steps 20 --top 60 > ${OUT}_summary.txt
python3 tools/rocpd_summary.py $DB --between spin_kernel --sequence 400 > ${OUT}_seq.txt
tail -3 ${OUT}.log
head -3 ${OUT}_summary.txt
rm -rf $OUT
