#!/bin/bash
# A/B of the prebuilt variant libraries (convolutionalencdec_amd/lib/exp/*): interleaved bench
# runs (HIP-event kernel ms) plus one tools/tstamp.py phase summary per variant.
# Usage (GPU box): bash tools/ab_tstamp.sh [reps] [extra bench.py / tstamp.py args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/abts; mkdir -p $o
reps=${1:-3}; shift
: > $o/ab.txt; : > $o/tstamp.jsonl
export TMPDIR=/tmp
for d in convolutionalencdec_amd/lib/exp/*/; do
  n=$(basename $d)
  VTB_LIB_PATH=$PWD/$d/libviterbi_amd.so timeout -k 10 120 python3 tools/tstamp.py "$@" > $o/ts_$n.json 2> $o/ts_$n.err || exit $?
  echo "{\"variant\": \"$n\", \"ts\": $(cat $o/ts_$n.json)}" >> $o/tstamp.jsonl
done
for r in $(seq $reps); do
  for d in convolutionalencdec_amd/lib/exp/*/; do
    n=$(basename $d)
    VTB_LIB_PATH=$PWD/$d/libviterbi_amd.so timeout -k 10 120 python3 bench.py --steps 100 --warmup 10 --cpu-seconds 0 "$@" > $o/ab_$n.log 2> $o/ab_$n.err || exit $?
    echo "$n $(grep -o '"kernel_avg_ms": [0-9.]*' $o/ab_$n.log | cut -d' ' -f2) $(grep -o '"value": [0-9.]*' $o/ab_$n.log | cut -d' ' -f2)" >> $o/ab.txt
  done
done
sort $o/ab.txt
