set -o pipefail
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for v in "X=0" "HYDRA_CAPTURE_PRIORITY=-1 HYDRA_SIDE_PRIORITY=-1" "X=0"; do
  env $v timeout -k 10 200 python bench.py --steps 40 --warmup 5 > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/ab.log | cut -c1-170)"
done
