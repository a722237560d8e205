#!/bin/bash
# Round 3: split fix-up check -- GPU suite, then split statistics with and without the fix-up
# (VTB_DEBUG bit 14) for every channel point, the persistent split kernel forced (k7s) and the
# library's own choice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/r03; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $o/fix_gpu_tests.log 2>&1 || { tail -30 $o/fix_gpu_tests.log; exit 1; }
tail -2 $o/fix_gpu_tests.log
VTB_KERNEL=k7s timeout -k 10 300 python3 tools/split_stats.py > $o/split_stats_fix.jsonl 2>&1 || exit 1
VTB_KERNEL=k7s VTB_DEBUG=16384 timeout -k 10 300 python3 tools/split_stats.py > $o/split_stats_nofix.jsonl 2>&1 || exit 1
timeout -k 10 300 python3 tools/split_stats.py > $o/split_stats_default.jsonl 2>&1 || exit 1
cat $o/split_stats_fix.jsonl $o/split_stats_nofix.jsonl $o/split_stats_default.jsonl
