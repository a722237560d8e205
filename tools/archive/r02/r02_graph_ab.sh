#!/bin/bash
# A/B on one box, the driver's command (--steps 20 --warmup 5): plain launches vs the K steps
# captured as one hipGraph (--graph); four interleaved rounds, then 50 steps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
o=gpurun_out/r02graph; mkdir -p $o
run() {
  local tag=$1; shift
  timeout -k 10 120 python3 bench.py --cpu-seconds 0 "$@" > $o/$tag.json 2> $o/$tag.err || { tail -5 $o/$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('$o/$tag.json')); r=d['roofline']; print('$tag', round(d['value']), d['ms_per_step'], r['kernel_ms'], r['per_launch_pass_ms']['median'])"
}
for r in 1 2 3 4; do
  run plain_s20_$r --steps 20 --warmup 5
  run graph_s20_$r --steps 20 --warmup 5 --graph
done
run plain_s50 --steps 50 --warmup 5; run graph_s50 --steps 50 --warmup 5 --graph
run plain_s20_hard --steps 20 --warmup 5 --hard; run graph_s20_hard --steps 20 --warmup 5 --hard --graph
exit 0
