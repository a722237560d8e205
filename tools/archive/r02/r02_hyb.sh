#!/bin/bash
# Round 2: hybrid survivors (global + newest steps in LDS) for the K=7 global-survivor variant:
# parity (gws family, C3 full batch), then C3 A/B against the pure-global variant
# (VTB_DEBUG=2048), and the speedDecode harness.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
o=gpurun_out/r02hyb; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ber.py tests/test_gpu_frame_sync.py -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > $o/tests.log 2>&1 || { tail -40 $o/tests.log; exit 1; }
tail -2 $o/tests.log
: > $o/ab.txt
for r in 1 2; do
  for d in 0 2048; do
    VTB_DEBUG=$d timeout -k 10 200 python3 bench.py --frames 65536 --frame-bits 2048 --steps 20 --warmup 3 --cpu-seconds 0 > $o/c3_$d.json 2> $o/c3_$d.err || exit $?
    echo "C3 soft debug=$d $(python3 -c "import json;d=json.load(open('$o/c3_$d.json'));print(d['value'], d['roofline']['kernel_ms'])")" >> $o/ab.txt
    VTB_DEBUG=$d timeout -k 10 200 python3 bench.py --frames 65536 --frame-bits 2048 --hard --steps 20 --warmup 3 --cpu-seconds 0 > $o/c3h_$d.json 2> $o/c3h_$d.err || exit $?
    echo "C3 hard debug=$d $(python3 -c "import json;d=json.load(open('$o/c3h_$d.json'));print(d['value'], d['roofline']['kernel_ms'])")" >> $o/ab.txt
  done
done
cat $o/ab.txt
timeout -k 10 60 bash tools/speed_decode.sh 5 > $o/speed_decode.txt 2>&1 || exit $?
cat $o/speed_decode.txt
exit 0
