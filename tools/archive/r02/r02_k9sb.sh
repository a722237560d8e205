#!/bin/bash
# Round 2: streaming bench, K=9 and K=7, soft and hard, 4096 streams x 1008 segments per call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
o=gpurun_out/r02k9sb; mkdir -p $o
export TMPDIR=/tmp
: > $o/stream_bench.jsonl
for k in 9 7; do for h in "" "--hard"; do
  timeout -k 10 200 python3 bench.py --K $k $h --stream-chunk 1008 --steps 20 --warmup 3 --cpu-seconds 0 >> $o/stream_bench.jsonl 2> $o/err_$k$h.log || exit $?
done; done
cat $o/stream_bench.jsonl | cut -c1-400
exit 0
