#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for sp in 0 1 2 4 8 16; do
  echo "== HYDRA_MM_SPLIT=$sp"
  if [ $sp -eq 0 ]; then timeout -k 10 120 python tools/bench_mm.py || exit $?; else HYDRA_MM_SPLIT=$sp timeout -k 10 120 python tools/bench_mm.py || exit $?; fi
done
