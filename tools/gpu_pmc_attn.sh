#!/bin/bash
# PMC counters of the attention kernels in the headline step (one counter pass)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/pmc_attn
rm -rf $OUT
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-include-regex "attn_(fwd_sk|bwd_dq|bwd_dkv)" --output-format csv -d $OUT -o run -- python3 bench.py --steps 3 --warmup 2 > ${OUT}.log 2>&1 || exit $?
find $OUT -name "*counter_collection*" | head -3
