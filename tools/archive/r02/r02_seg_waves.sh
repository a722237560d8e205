#!/bin/bash
# K=7 single-frame kernel: waves per workgroup (up to 8 = two per SIMD) x warm-up, speedDecode
# (4 s per point), then the frame-sync tests at 8 waves.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
o=gpurun_out/r02segw; mkdir -p $o
for w in 4 5 6 8; do for m in 96 48; do
  VTB_SEG_WAVES=$w VTB_SEG_WARM=$m oracle/_ref/speedDecode_amd > $o/w$w-m$m.log 2>&1 &
  pid=$!; sleep 5; kill $pid; wait $pid 2>/dev/null
  echo "waves=$w warm=$m $(grep -h Rate $o/w$w-m$m.log | tail -2 | sed 's/.*Rate: //' | tr '\n' ' ')"
done; done
VTB_SEG_WAVES=8 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_frame_sync.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $o/tests8.log 2>&1 || { tail -30 $o/tests8.log; exit 1; }
tail -1 $o/tests8.log
exit 0
