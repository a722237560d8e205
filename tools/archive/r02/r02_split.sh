#!/bin/bash
# Round 2: persistent split kernel for long K=7 frames: parity (every family incl. k7s, C3 full
# batch, fuzz), then C3 soft / hard A/B against the global-survivor variant (VTB_DEBUG=4096).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
o=gpurun_out/r02split; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 800 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ber.py tests/test_gpu_fuzz.py tests/test_gpu_multi.py -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
: > $o/ab.txt
for r in 1 2; do
  for d in 0 4096; do
    for h in "" "--hard"; do
      VTB_DEBUG=$d timeout -k 10 200 python3 bench.py --frames 65536 --frame-bits 2048 $h --gen device --steps 20 --warmup 3 --cpu-seconds 0 > $o/c3.json 2> $o/c3.err || exit $?
      echo "C3 $h debug=$d $(python3 -c "import json;d=json.load(open('$o/c3.json'));print(d['value'], d['roofline']['kernel_ms'], d['config']['decoded_ber'])")" >> $o/ab.txt
    done
  done
done
cat $o/ab.txt
exit 0
