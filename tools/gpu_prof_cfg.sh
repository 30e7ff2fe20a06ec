#!/bin/bash
# rocprofv3 per-step kernel summary of one bench_configs config: $1 = config, $2 = precision
# (the timed steps are bracketed by spin kernels; the summary covers exactly those steps)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HYDRA_PROFILE_MARK=1
OUT=gpurun_out/prof_cfg_$1_$2
rm -rf $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --output-format rocpd -d $OUT -o run -- python3 tools/bench_configs.py $1 --steps 10 --warmup 5 --precision $2 > ${OUT}.log 2>&1 || exit $?
DB=$(find $OUT -name "*.db" | head -1)
python3 tools/rocpd_summary.py $DB --between spin_kernel --steps 10 --top 40 > ${OUT}_summary.txt
grep metric ${OUT}.log | cut -c1-200
head -30 ${OUT}_summary.txt | cut -c1-160
rm -rf $OUT  # the trace db stays on the box (gpurun_out is copied back only under 64 MiB)
