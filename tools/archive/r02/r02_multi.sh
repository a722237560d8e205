#!/bin/bash
# Round 2: multi-GPU paths on one GPU (peer scatter staged, host multi) and the C5 shard.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
o=gpurun_out/r02multi; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_multi.py -x -v -p no:cacheprovider --timeout 240 --timeout-method thread > $o/tests.log 2>&1 || { tail -40 $o/tests.log; exit 1; }
tail -25 $o/tests.log
exit 0
