#!/bin/bash
# Counter passes (kernel trace only) over an arbitrary short command:
#   PMC_NAME=<dir name> tools/gpu_pmc_cmd.sh python3 <script> [args]
# pass A: issue / wait / MFMA-busy cycles, pass B: instruction mix, pass C: L2 / EA traffic.
# Summary: tools/pmc_roofline.py -> gpurun_out/<name>_summary.txt
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
NAME=${PMC_NAME:-pmc_cmd}
OUT=gpurun_out/$NAME
rm -rf $OUT
mkdir -p $OUT
run_pass() {  # name counters... (the command follows --)
  local name=$1; shift
  timeout -s KILL 180 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $OUT/$name -o run -- \
    "${CMD[@]}" > $OUT/$name.log 2>&1
}
CMD=("$@")
run_pass A SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT || exit $?
run_pass B SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU \
  SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_MFMA_MOPS_F32 || exit $?
run_pass C TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum || exit $?
python3 tools/pmc_roofline.py $OUT > gpurun_out/${NAME}_summary.txt 2>&1
head -30 gpurun_out/${NAME}_summary.txt
