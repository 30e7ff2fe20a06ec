#!/bin/bash
# attention8 iteration: GPU tests, timing sweep, one PMC pass over the sweep's kernels
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention8_gpu.py > gpurun_out/t_attn8.log 2>&1 || { tail -30 gpurun_out/t_attn8.log; exit 1; }
tail -2 gpurun_out/t_attn8.log
timeout -k 10 120 python tools/bench_attn8.py 2560 2311 > gpurun_out/attn8_v2.log 2>&1 || exit 1
cat gpurun_out/attn8_v2.log
rm -rf gpurun_out/pmc_attn8
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --kernel-trace --kernel-include-regex "attn8_(fwd2|bwd2)" \
  --output-format csv -d gpurun_out/pmc_attn8/A -o run -- python3 tools/bench_attn8.py 2560 2311 > gpurun_out/pmc_attn8.log 2>&1 || exit 1
python3 tools/pmc_roofline.py gpurun_out/pmc_attn8 > gpurun_out/pmc_attn8_summary.txt 2>&1
head -14 gpurun_out/pmc_attn8_summary.txt
# head+loss kernels: device time per launch from the kernel trace (the event timing of
# tools/bench_head_loss.py is host-bound)
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --kernel-include-regex "head_loss" --output-format csv \
  -d gpurun_out/prof_hl -o run -- python3 tools/bench_head_loss.py > gpurun_out/prof_hl.log 2>&1 || exit 1
find gpurun_out/prof_hl -name "*kernel_stats*" -exec cat {} \;
