#!/bin/bash
# Round 2: general-k decoder parity and throughput (tools/genk_bench.py) + rocprof stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
o=gpurun_out/r02genk; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_genk.py tests/test_gpu_legacy.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
timeout -k 10 200 python3 tools/genk_bench.py > $o/genk_bench.jsonl 2> $o/genk_bench.err || exit $?
cat $o/genk_bench.jsonl
exit 0
