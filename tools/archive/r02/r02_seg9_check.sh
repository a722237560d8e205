#!/bin/bash
# Round 2: the full GPU suite and three 2,000-case fuzz sweeps (single-frame path incl. K=9
# over several workgroups) after the stream-ordered SEG counter zeroing and the split-tail fix.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
o=gpurun_out/seg9check; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $o/gpu_tests.log 2>&1 || { tail -30 $o/gpu_tests.log; exit 1; }
tail -1 $o/gpu_tests.log
VTB_FUZZ_N=2000 timeout -k 10 900 bash tools/r02_fuzz_long.sh 31337 2026 99991 || exit 1
exit 0
