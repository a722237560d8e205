#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
o=gpurun_out/r02parity; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -rs -p no:cacheprovider --timeout 300 --timeout-method thread > $o/tests.log 2>&1 || { tail -40 $o/tests.log; exit 1; }
grep -E "^SKIPPED" $o/tests.log | sed 's/\[[0-9]*\]//' | sort | uniq -c | sort -rn | head -20
tail -1 $o/tests.log
