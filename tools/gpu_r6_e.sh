set -o pipefail
cd $GRAFT_REPO_ROOT
run() { timeout -k 10 "$@"; rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc; }
for cfg in "4 512" "4 256" "2 256" "2 512" "1 256"; do
set -- $cfg
HYDRA_ROWPROG_ROWS=$1 HYDRA_ROWPROG_THREADS=$2 run 300 python tools/bench_configs.py md17_painn_forces --steps 30 --warmup 5 > gpurun_out/b5.log 2>&1; echo "rows=$1 nt=$2 $(grep metric gpurun_out/b5.log | cut -c1-160)"
done
