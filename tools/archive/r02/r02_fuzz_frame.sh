#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
o=gpurun_out/r02fuzz; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_fuzz.py tests/test_gpu_frame_sync.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
