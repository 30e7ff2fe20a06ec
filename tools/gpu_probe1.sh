set -o pipefail
cd $GRAFT_REPO_ROOT
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
echo "== 1 rank probe"; timeout -k 10 120 $TR --nproc-per-node 1 --master-port 29511 tools/rccl_probe.py > gpurun_out/probe_1r.log 2>&1; echo "rc=$?"; tail -5 gpurun_out/probe_1r.log
echo "== bench 1 GPU"; timeout -k 10 180 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_1.log 2>&1; echo "rc=$?"; tail -2 gpurun_out/bench_1.log
echo "== bench 1 rank torchrun forced captured sync"; HYDRA_GRADSYNC_FORCE=1 timeout -k 10 180 $TR --nproc-per-node 1 --master-port 29512 bench.py --steps 20 --warmup 5 > gpurun_out/bench_1r_sync.log 2>&1; echo "rc=$?"; tail -2 gpurun_out/bench_1r_sync.log
echo "== 2 ranks same GPU probe"; timeout -k 10 90 $TR --nproc-per-node 2 --master-port 29513 tools/rccl_probe.py > gpurun_out/probe_2r.log 2>&1; echo "rc=$?"; tail -8 gpurun_out/probe_2r.log
