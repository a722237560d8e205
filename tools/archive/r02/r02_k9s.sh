#!/bin/bash
# Round 2: K=9 streaming parity (and the K=7 streaming suite, unchanged kernel).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
o=gpurun_out/r02k9s; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_stream_k9.py tests/test_gpu_stream.py -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > $o/tests.log 2>&1 || { tail -40 $o/tests.log; exit 1; }
tail -5 $o/tests.log
exit 0
