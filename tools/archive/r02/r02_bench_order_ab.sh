#!/bin/bash
# A/B of bench.py's order (output check before the timed region = bench_prev.py, after it =
# bench.py) on the driver's exact command, interleaved rounds on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
o=gpurun_out/order_ab; mkdir -p $o; : > $o/summary.txt
for r in 1 2 3 4 5; do
  for b in bench_prev bench; do  # (bench_prev.py: a copy of the previous bench.py, not kept)
    timeout -k 10 300 python3 $b.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 > $o/${b}_$r.json 2> $o/${b}_$r.err || exit 1
    python3 -c "import json; d=json.load(open('$o/${b}_$r.json')); print('$b', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])" >> $o/summary.txt
  done
done
sort $o/summary.txt
