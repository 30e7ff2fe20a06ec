#!/bin/bash
# Standalone attention timing at the OC20 bench shape + one PMC pass over the fwd/bwd kernels
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/bench_attn.py 2311 8 8 > gpurun_out/attn_time.log 2>&1 || exit $?
cat gpurun_out/attn_time.log
OUT=gpurun_out/pmc_attn2
rm -rf $OUT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-include-regex "attn_(fwd_sk|bwd_dq|bwd_dkv)" --output-format csv -d $OUT -o run -- python3 tools/bench_attn.py 2311 8 8 > ${OUT}.log 2>&1 || exit $?
f=$(find $OUT -name "*counter_collection.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].split("(")[0][-40:]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"]); cnt[(k, r["Counter_Name"])] += 1
for k, d in agg.items():
    n = cnt[(k, "SQ_WAVES")] or 1
    print(k, {c: round(v / n) for c, v in d.items()})
PY
