#!/bin/bash
# K=9 single-frame kernel phases: kernel durations with everything, without the traceback
# (VTB_DEBUG=1) and without ACS and traceback (3); then the frame tests and speedDecode.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
o=gpurun_out/r02ph9; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_frame_sync.py tests/test_gpu_legacy.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
for dbg in 0 1 3; do for K in 7 9; do
  VTB_DEBUG=$dbg timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $o/p$dbg-$K -o run -- python3 tools/probes/frame_phases.py $K 2048 3000 > $o/p$dbg-$K.log 2>&1 || { cat $o/p$dbg-$K.log; exit 1; }
  echo "dbg=$dbg K=$K: $(grep us $o/p$dbg-$K.log)"
  f=$(ls $o/p$dbg-$K/*/run_kernel_stats.csv 2>/dev/null || ls $o/p$dbg-$K/run_kernel_stats.csv)
  grep -h "seg" $f | cut -c1-200
done; done
timeout -k 10 90 bash tools/speed_decode.sh 4 k9 > $o/speed_decode.txt 2>&1 || exit $?
cat $o/speed_decode.txt
exit 0
