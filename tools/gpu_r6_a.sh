set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_head_loss_gpu.py tests/test_gradslots.py tests/test_egnn_wide_gpu.py > gpurun_out/t1.log 2>&1; tail -2 gpurun_out/t1.log
timeout -k 10 300 python tools/overlap_check.py --config multibranch_egnn --precision bf16 > gpurun_out/ov.log 2>&1 || { tail -20 gpurun_out/ov.log; exit 1; }
tail -1 gpurun_out/ov.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['bytes_overlapped_fraction'], d['launches_after_each_allreduce'])"
tail -1 gpurun_out/ov.log > gpurun_out/overlap_egnn_bf16.json
timeout -k 10 200 python bench.py --steps 50 --warmup 10 > gpurun_out/b1.log 2>&1 || exit 1
cut -c1-150 gpurun_out/b1.log
timeout -k 10 300 bash tools/gpu_prof_headline_final.sh > gpurun_out/prof.log 2>&1 || exit 1
cat gpurun_out/prof.log
