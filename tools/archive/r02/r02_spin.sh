#!/bin/bash
# Round 2: A/B of the host wait mode around the driver's bench command.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
o=gpurun_out/r02spin; mkdir -p $o
export TMPDIR=/tmp
: > $o/ab.txt
for r in 1 2 3; do
  for m in spin auto; do
    timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --sync $m > $o/b_$m.json 2> $o/b_$m.err || exit $?
    echo "$m $(python3 -c "import json;d=json.load(open('$o/b_$m.json'));print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['host_issue_us_per_launch'])")" >> $o/ab.txt
  done
done
cat $o/ab.txt
exit 0
