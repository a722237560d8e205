#!/bin/bash
# K=9 single frame with the adaptive warm-up: workgroups (VTB_SEG9_WGS), 4 s per point.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
o=gpurun_out/r02sd9g; mkdir -p $o
for g in 3 4 6 8 12; do
  VTB_SEG9_WGS=$g oracle/_ref/speedDecode_amd_k9 > $o/g$g.log 2>&1 &
  pid=$!; sleep 5; kill $pid; wait $pid 2>/dev/null
  echo "wgs=$g $(grep -h Rate $o/g$g.log | tail -2 | sed 's/.*Rate: //' | tr '\n' ' ')"
done
exit 0
