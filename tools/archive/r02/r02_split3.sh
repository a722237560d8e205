#!/bin/bash
# Measurement only: persistent split kernel on C3 shapes with a 96-step warm-up (7 waves per
# CU) vs the default choice, soft and hard.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
o=gpurun_out/r02split3; mkdir -p $o
export TMPDIR=/tmp
VTB_KERNEL=k7s VTB_SPLIT_WARM=96 timeout -k 10 300 python3 tools/split_stats.py > $o/w96.jsonl 2> $o/w96.err || exit $?
VTB_KERNEL=k7s timeout -k 10 300 python3 tools/split_stats.py > $o/w48.jsonl 2> $o/w48.err || exit $?
timeout -k 10 300 python3 tools/split_stats.py > $o/auto.jsonl 2> $o/auto.err || exit $?
cat $o/w96.jsonl $o/w48.jsonl $o/auto.jsonl
exit 0
