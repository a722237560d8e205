#!/bin/bash
# Round 2 split-half tail fix: the new regression tests against the previous library
# (convolutionalencdec_amd/lib/exp/base, built before the fix: expected to fail), then the full
# GPU suite, the fuzz case that found it, and the fuzz sweep that found it, on the fixed library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
o=gpurun_out/splitfix; mkdir -p $o
export TMPDIR=/tmp
if [ -f convolutionalencdec_amd/lib/exp/base/libviterbi_amd.so ]; then
  VTB_LIB_PATH=$PWD/convolutionalencdec_amd/lib/exp/base/libviterbi_amd.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -k "split_frames or split_loop_odd" -q -p no:cacheprovider --timeout 120 --timeout-method thread > $o/old_lib_new_tests.log 2>&1
  echo "old library, new split tests: exit $? ($(tail -1 $o/old_lib_new_tests.log))"
fi
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $o/gpu_tests.log 2>&1 || { tail -30 $o/gpu_tests.log; exit 1; }
tail -1 $o/gpu_tests.log
timeout -k 10 120 python3 tools/dbg_frame_case.py > $o/case1947.jsonl 2> $o/case1947.err || exit 1
cat $o/case1947.jsonl
VTB_FUZZ_N=2000 timeout -k 10 900 bash tools/r02_fuzz_long.sh 31337 2026 || exit 1
exit 0
