#!/bin/bash
# Roofline counters of the hot kernels of the headline step (bench.py), one counter set per
# rocprofv3 pass (kernel trace only, never combined with the runtime/sys trace domains):
#   pass A: issue / wait / MFMA-busy cycles   pass B: instruction mix   pass C: HBM bytes (EA)
# Summary: tools/pmc_roofline.py -> gpurun_out/pmc_top_summary.txt
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/pmc_top
rm -rf $OUT
mkdir -p $OUT
ARGS=${PMC_BENCH_ARGS:-"--steps 4 --warmup 2"}
timeout -s KILL 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
have() { grep -q "$1" $OUT/counters_list.txt; }
run_pass() {  # name counters...
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $OUT/$name -o run -- \
    python3 bench.py $ARGS > $OUT/$name.log 2>&1
}
run_pass A SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT || exit $?
B=""
for c in SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU \
         SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_MFMA_MOPS_F32; do
  have "$c" && B="$B $c"
done
run_pass B $B || exit $?
C=""
for c in TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum; do
  have "${c%_sum}" && C="$C $c"
done
[ -n "$C" ] && { run_pass C $C TCC_HIT_sum TCC_MISS_sum || exit $?; }
python3 tools/pmc_roofline.py $OUT > gpurun_out/pmc_top_summary.txt 2>&1
cat gpurun_out/pmc_top_summary.txt | head -80
