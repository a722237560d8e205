#!/bin/bash
# Round 2: where the hybrid-survivor C3 soft launch loses time: ACS only (VTB_DEBUG bit 0 skips
# the traceback) for hybrid vs pure global (bit 11).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
o=gpurun_out/r02hyb2; mkdir -p $o
export TMPDIR=/tmp
: > $o/ab.txt
for r in 1 2; do
  for d in 1 2049 0 2048; do
    VTB_DEBUG=$d timeout -k 10 200 python3 bench.py --frames 65536 --frame-bits 2048 --steps 20 --warmup 3 --cpu-seconds 0 --gen device > $o/c3_$d.json 2> $o/c3_$d.err || exit $?
    echo "C3 soft debug=$d $(python3 -c "import json;d=json.load(open('$o/c3_$d.json'));print(d['value'], d['roofline']['kernel_ms'])")" >> $o/ab.txt
  done
done
cat $o/ab.txt
exit 0
