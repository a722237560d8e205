#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
o=gpurun_out/r02sd8; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_frame_sync.py tests/test_gpu_legacy.py tests/test_gpu_fuzz.py -k "not random_case" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
timeout -k 10 90 bash tools/speed_decode.sh 5 k9 > $o/speed_decode.txt 2>&1 || exit $?
cat $o/speed_decode.txt
exit 0
