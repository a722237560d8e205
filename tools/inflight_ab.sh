#!/bin/bash
# Batches in flight A/B on the driver's command form: interleaved reps of
#   bench.py --steps S --warmup 5 --inflight N   (N from the arguments)
# Prints "inflight steps ms_per_step value kernel_ms" per run into gpurun_out/inflight_ab.txt.
# Usage (GPU box): bash tools/inflight_ab.sh <reps> <steps> <n> [<n> ...] [-- extra bench args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
reps=$1 steps=$2; shift 2
ns=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do ns+=("$1"); shift; done
[ "$1" = "--" ] && shift
out=gpurun_out/inflight_ab.txt; : > $out
for r in $(seq $reps); do
  for n in "${ns[@]}"; do
    timeout -k 10 120 python3 bench.py --steps $steps --warmup 5 --cpu-seconds 0 --inflight $n "$@" > gpurun_out/inflight_$n.json 2> gpurun_out/inflight_$n.err || exit $?
    python3 - "$n" "$steps" gpurun_out/inflight_$n.json >> $out <<'EOF'
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
print(sys.argv[1], sys.argv[2], d["ms_per_step"], d["value"], d["roofline"]["kernel_avg_ms"])
EOF
  done
done
sort -n $out
