#!/bin/bash
# A/B timing of the prebuilt variant libraries (convolutionalencdec_amd/lib/exp/*), interleaved
# over several repetitions to average out clock drift.  Prints kernel ms (HIP events) per run.
# Usage (GPU box): bash tools/ab_variants.sh [reps] [extra bench.py args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
reps=${1:-3}; shift
out=gpurun_out/ab.txt; : > $out
for r in $(seq $reps); do
  for d in ${VARIANTS:-convolutionalencdec_amd/lib/exp/*/}; do  # $VARIANTS: a subset (dirs)
    n=$(basename $d)
    VTB_LIB_PATH=$PWD/$d/libviterbi_amd.so timeout -k 10 120 python bench.py --steps 100 --warmup 10 --cpu-seconds 0 "$@" > gpurun_out/ab_$n.log 2>&1 || exit $?
    echo "$n $(grep -o '"kernel_avg_ms": [0-9.]*' gpurun_out/ab_$n.log | cut -d' ' -f2) $(grep -o '"value": [0-9.]*' gpurun_out/ab_$n.log | cut -d' ' -f2)" >> $out
  done
done
sort $out
