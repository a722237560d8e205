#!/bin/bash
# SEG kernel geometry sweep on the reference speedDecode harness (legacy drop-in, one frame
# per call): VTB_SEG_WAVES x VTB_SEG_WARM, 4 s each, the last per-second rate.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/segsweep; mkdir -p $o
: > $o/sweep.txt
for w in 4 3 2; do
  for m in 96 48; do
    VTB_SEG_WAVES=$w VTB_SEG_WARM=$m oracle/_ref/speedDecode_amd > $o/run_${w}_${m}.log 2>&1 &
    pid=$!; sleep 4; kill $pid; wait $pid 2>/dev/null
    echo "waves $w warm $m: $(grep Rate $o/run_${w}_${m}.log | tail -1)" >> $o/sweep.txt
  done
done
VTB_DEBUG=1024 oracle/_ref/speedDecode_amd > $o/run_noseg.log 2>&1 &
pid=$!; sleep 4; kill $pid; wait $pid 2>/dev/null
echo "no SEG (split frame kernel): $(grep Rate $o/run_noseg.log | tail -1)" >> $o/sweep.txt
cat $o/sweep.txt
exit 0
