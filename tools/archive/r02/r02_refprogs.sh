#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
o=gpurun_out/r02ref; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_legacy.py -k "reference or handtraced" -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $o/tests.log 2>&1 || { tail -40 $o/tests.log; exit 1; }
tail -4 $o/tests.log
timeout -k 10 120 oracle/_ref/handTraced_amd > $o/handTraced.txt 2>&1; echo "handTraced exit $?"
( time timeout -k 10 300 oracle/_ref/berTestK7_amd ) > $o/berTestK7.txt 2>&1 || exit 1
tail -12 $o/berTestK7.txt
