#!/bin/bash
# Measurement: the driver's bench command at several step counts (fixed per-region overhead vs
# per-launch time), two rounds interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04; o=gpurun_out/r04/steps_sweep.txt; : > $o
for r in 1 2; do
  for k in 1 5 20 100; do
    timeout -k 10 120 python3 bench.py --steps $k --warmup 5 --cpu-seconds 0 > gpurun_out/steps_$k.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/steps_$k.json')); r=d['roofline']; print($k, d['ms_per_step'], r['kernel_avg_ms'], r['timed_span_ms'], r['host_issue_us_per_launch'])" >> $o
  done
done
cat $o
