#!/bin/bash
# Round-2 confirmation after the last library change: full GPU suite, smoke, the driver's
# bench command, the speedDecode / speedEncode harnesses.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
o=gpurun_out/r02confirm; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $o/gpu_tests.log 2>&1 || { tail -30 $o/gpu_tests.log; exit 1; }
tail -1 $o/gpu_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit 1
tail -1 $o/smoke.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $o/bench.json 2> $o/bench.err || exit 1
python3 -c "import json; d=json.load(open('$o/bench.json')); r=d['roofline']; print('bench', d['value'], r['kernel_ms'], r['frac'], r['traffic'], r['secondary'].get('frac'), d['cpu_baseline']['value'])"
timeout -k 10 90 bash tools/speed_decode.sh 4 k9 > $o/speed_decode.txt 2>&1 || exit 1
cat $o/speed_decode.txt
exit 0
