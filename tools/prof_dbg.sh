#!/bin/bash
# Kernel-trace durations of the default bench workload with VTB_DEBUG = 0 (full), 1 (ACS
# only), 3 (neither ACS nor traceback: prologue/epilogue only).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for d in ${PROF_DBG_LIST:-0 1 3}; do
  rm -rf gpurun_out/prof_dbg$d
  VTB_DEBUG=$d timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_dbg$d -o run -- python3 bench.py --steps 20 --warmup 2 --cpu-seconds 0 > gpurun_out/prof_dbg$d.log 2>&1 || exit $?
done
exit 0
