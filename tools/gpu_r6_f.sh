set -o pipefail
cd $GRAFT_REPO_ROOT
run() { timeout -k 10 "$@"; rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc; }
for i in 1 2; do for v in 1 0; do
HYDRA_FCN_LINACT=$v run 300 python tools/bench_configs.py multibranch_mace --steps 40 --warmup 5 > gpurun_out/b6.log 2>&1; echo "linact=$v $(grep metric gpurun_out/b6.log | cut -c1-150)"
done; done
