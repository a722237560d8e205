#!/bin/bash
# K=9 single frame (speedDecode, params/k9): waves per workgroup x workgroups, 4 s per point;
# then the K=9 frame tests at 8 waves.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
o=gpurun_out/r02sd9w; mkdir -p $o
export TMPDIR=/tmp
for w in 4 8; do for g in 1 2 3 4 6; do
  VTB_SEG9_WAVES=$w VTB_SEG9_WGS=$g oracle/_ref/speedDecode_amd_k9 > $o/w$w-g$g.log 2>&1 &
  pid=$!; sleep 5; kill $pid; wait $pid 2>/dev/null
  echo "waves=$w wgs=$g $(grep -h Rate $o/w$w-g$g.log | tail -2 | sed 's/.*Rate: //' | tr '\n' ' ')"
done; done
VTB_SEG9_WAVES=8 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_frame_sync.py -k k9 -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $o/tests8.log 2>&1 || { tail -30 $o/tests8.log; exit 1; }
tail -1 $o/tests8.log
exit 0
