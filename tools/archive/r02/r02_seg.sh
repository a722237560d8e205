#!/bin/bash
# Round 2: the single-frame SEG path -- its parity tests, then the reference speedDecode
# harness against the legacy drop-in.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
o=gpurun_out/r02seg; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_frame_sync.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > $o/tests.log 2>&1 || { tail -40 $o/tests.log; exit 1; }
tail -3 $o/tests.log
timeout -k 10 60 bash tools/speed_decode.sh 5 > $o/speed_decode.txt 2>&1 || exit $?
cat $o/speed_decode.txt
exit 0
