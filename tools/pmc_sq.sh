#!/bin/bash
# SQ counter passes (issue / wait breakdown) on the default bench workload.  Each pass is a
# separate rocprofv3 run with --pmc and --kernel-trace only.
# Usage: bash tools/pmc_sq.sh [VTB_DEBUG value]   (1 = ACS only)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
dbg=${1:-0}
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE" \
           "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS SQ_INST_CYCLES_SMEM" \
           "SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_INSTS SQ_ACTIVE_INST_VALU2 SQ_INST_LEVEL_SMEM SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  rm -rf gpurun_out/pmc_sq$i
  VTB_DEBUG=$dbg timeout -k 10 300 rocprofv3 --pmc $set --kernel-trace --output-format csv -d gpurun_out/pmc_sq$i -o run -- python3 bench.py --steps 10 --warmup 2 --cpu-seconds 0 ${PMC_BENCH_ARGS:-} > gpurun_out/pmc_sq$i.log 2>&1 || exit $?
done
exit 0
