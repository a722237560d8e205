#!/bin/bash
# Round 2: fuzz sweep (incl. the single-frame path and the hard hybrid variant), general-k
# parity and throughput.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
o=gpurun_out/r02fuzz; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fuzz.py tests/test_gpu_genk.py tests/test_gpu_legacy.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
timeout -k 10 200 python3 tools/genk_bench.py > $o/genk_bench.jsonl 2> $o/genk_bench.err || exit $?
cat $o/genk_bench.jsonl
exit 0
