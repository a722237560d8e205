#!/bin/bash
# A/B timing of runtime switches (environment variables) on one library, interleaved over
# several repetitions to average out clock drift.  Prints "label kernel_ms Mbit/s" per run.
# Usage (GPU box): bash tools/ab_env.sh <reps> "<label>=<VAR=value ...>" ... -- [bench.py args]
#   bash tools/ab_env.sh 4 "trim=" "full=VTB_DEBUG=8192" -- --hard
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
reps=$1; shift
arms=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do arms+=("$1"); shift; done
[ "$1" = "--" ] && shift
out=gpurun_out/ab_env.txt; : > $out
for r in $(seq $reps); do
  for a in "${arms[@]}"; do
    label=${a%%=*}; vars=${a#*=}
    env $vars timeout -k 10 120 python3 bench.py --steps 100 --warmup 10 --cpu-seconds 0 "$@" > gpurun_out/ab_env_$label.log 2>&1 || exit $?
    echo "$label $(grep -o '"kernel_avg_ms": [0-9.]*' gpurun_out/ab_env_$label.log | cut -d' ' -f2) $(grep -o '"value": [0-9.]*' gpurun_out/ab_env_$label.log | cut -d' ' -f2)" >> $out
  done
done
sort $out
