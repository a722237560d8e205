#!/bin/bash
# Round 2: where a 4096-frame launch goes -- per-wave timestamps (tools/tstamp.py) and
# rocprofv3 kernel durations of the VTB_DEBUG phase variants (16: return at entry, 3: no ACS
# and no traceback, 1: no traceback, 0: full).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
o=gpurun_out/r02phase; mkdir -p $o
export TMPDIR=/tmp
for args in "" "--hard" "--frames 8192" "--frames 2048" "--frames 65536"; do
  timeout -k 10 120 python3 tools/tstamp.py $args >> $o/tstamp.jsonl 2>> $o/tstamp.err || exit $?
done
for d in 16 3 1 0; do
  rm -rf $o/prof_d$d
  VTB_DEBUG=$d timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof_d$d -o run -- python3 bench.py --steps 50 --warmup 5 --cpu-seconds 0 > $o/bench_d$d.json 2> $o/bench_d$d.err || exit $?
done
exit 0
