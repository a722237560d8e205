#!/bin/bash
# Where the headline launch's wave cycles go (SQ counters, one rocprofv3 pass each;
# SQ_* in quad-cycles).  Measurement only.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/stalls${TAG:+_$TAG}; mkdir -p $o  # TAG / BARGS: another workload
export TMPDIR=/tmp
i=0
for ctr in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_WAVES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INST_CYCLES_VMEM" \
           "SQ_WAVES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INST_LEVEL_LDS SQ_IFETCH SQ_INSTS_BRANCH"; do
  i=$((i+1))
  rm -rf $o/p$i
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $o/p$i -o run -- python3 bench.py --steps 10 --warmup 2 --cpu-seconds 0 $BARGS > $o/p$i.log 2>&1 || exit $?
done
exit 0
