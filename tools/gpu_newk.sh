#!/bin/bash
# new fused kernels: oracle tests, then the GPU end-to-end accuracy tests of the affected stacks
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-newk}
timeout -k 10 400 python -u -m pytest tests/test_fused_gpu.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_fused.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/${TAG}_fused.log | tail -8
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u -m pytest tests/test_graphs.py -m gpu -k "GAT or CGCNN or MFC or MACE" -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_graphs.log 2>&1
rc=$?
grep -E "passed|failed|FAILED" gpurun_out/${TAG}_graphs.log | tail -8
exit $rc
