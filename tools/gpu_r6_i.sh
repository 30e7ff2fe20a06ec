#!/bin/bash
# multi-rank rehearsal of the bench contract on the one-GPU box: 2 and 4 ranks sharing the
# card over gloo (RCCL refuses duplicate devices; the driver's N-GPU runs use RCCL)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export BENCH_BACKEND=gloo
for n in 2 4; do
  timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29500 + n)) bench.py --gpus $n --steps 10 --warmup 5 > gpurun_out/r6_bench_${n}rank_gloo.log 2>&1 || { tail -30 gpurun_out/r6_bench_${n}rank_gloo.log; exit 1; }
  grep metric gpurun_out/r6_bench_${n}rank_gloo.log | cut -c1-240
done
