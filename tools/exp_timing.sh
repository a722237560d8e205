#!/bin/bash
# Measurement experiments (outputs are not checked): ACS-only / TB-only timing of the reg path.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for d in 0 1 2 3; do
  VTB_DEBUG=$d timeout -k 10 120 python bench.py --steps 30 --warmup 3 --cpu-seconds 0 > gpurun_out/exp_dbg$d.log 2>&1 || exit $?
done
