#!/bin/bash
# Run a sequence of GPU steps on the gpurun box; stop at the first crash/timeout
# (exit codes other than 0/1).  Usage: tools/gpu_session.sh "name|timeout|cmd" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"; t="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== $name (timeout ${t}s): $cmd"
  timeout -k 10 "$t" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc"
  tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
done
exit 0
