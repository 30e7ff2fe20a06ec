set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/op_census.py multibranch_mace --top 60 > gpurun_out/census_mace.txt 2>&1 || exit 1
timeout -k 10 300 python tools/op_census.py qm9_dimenet --top 60 > gpurun_out/census_dimenet.txt 2>&1 || exit 1
timeout -k 10 400 bash tools/gpu_prof_cfg.sh qm9_dimenet fp32 > gpurun_out/prof_dimenet.log 2>&1 || exit 1
timeout -k 10 400 bash tools/gpu_prof_cfg.sh qm9_schnet fp32 > gpurun_out/prof_schnet.log 2>&1 || exit 1
timeout -k 10 400 bash tools/gpu_prof_cfg.sh multibranch_mace fp32 > gpurun_out/prof_mace.log 2>&1 || exit 1
head -3 gpurun_out/prof_dimenet.log gpurun_out/prof_schnet.log gpurun_out/prof_mace.log | cut -c1-200
