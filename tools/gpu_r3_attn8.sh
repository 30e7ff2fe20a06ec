#!/bin/bash
# MFMA attention (8-wide heads): numerics, microbench, fused encoder tests, headline bench + profile, PMC
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention8_gpu.py > gpurun_out/r3_attn8_tests.log 2>&1
rc=$?; tail -15 gpurun_out/r3_attn8_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 tools/bench_attn8.py > gpurun_out/r3_attn8_bench.log 2>&1 || exit $?
cat gpurun_out/r3_attn8_bench.log | grep -v amdgpu.ids
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gps_fused_gpu.py > gpurun_out/r3_fused_tests2.log 2>&1
rc=$?; tail -5 gpurun_out/r3_fused_tests2.log; [ $rc -eq 0 ] || exit $rc
HYDRA_STEP_TIMING=1 timeout -k 10 240 python3 bench.py --steps 50 --warmup 10 > gpurun_out/r3_attn8_headline.log 2>&1 || exit $?
tail -1 gpurun_out/r3_attn8_headline.log | cut -c1-500
bash tools/gpu_prof_bench.sh r3_attn8 || exit $?
OUT=gpurun_out/pmc_attn8; rm -rf $OUT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-include-regex "attn8" --output-format csv -d $OUT -o run -- python3 tools/bench_attn8.py > ${OUT}.log 2>&1 || exit $?
python3 tools/pmc_summary.py $OUT > gpurun_out/r3_attn8_pmc.txt 2>&1; cat gpurun_out/r3_attn8_pmc.txt
