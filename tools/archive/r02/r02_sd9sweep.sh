#!/bin/bash
# K=9 single-frame drop-in (speedDecode, params/k9): workgroup count and XCD-local placement
# of k9_seg_kernel, 4 s per point.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
o=gpurun_out/r02sd9; mkdir -p $o
for x in 0 1; do for w in 2 4 8 16; do
  VTB_SEG9_XCD=$x VTB_SEG9_WGS=$w oracle/_ref/speedDecode_amd_k9 > $o/x$x-w$w.log 2>&1 &
  pid=$!; sleep 5; kill $pid; wait $pid 2>/dev/null
  echo "xcd=$x wgs=$w $(grep -h Rate $o/x$x-w$w.log | tail -2 | sed 's/.*Rate: //' | tr '\n' ' ')"
done; done
exit 0
