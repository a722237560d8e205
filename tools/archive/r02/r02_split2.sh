#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
o=gpurun_out/r02split2; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/split_stats.py > $o/stats.jsonl 2> $o/stats.err || exit $?
VTB_DEBUG=4096 timeout -k 10 300 python3 tools/split_stats.py > $o/stats_gs.jsonl 2> $o/stats_gs.err || exit $?
cat $o/stats.jsonl $o/stats_gs.jsonl
exit 0
