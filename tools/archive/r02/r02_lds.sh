#!/bin/bash
# Round 2: generic LDS-path kernel with the block-parallel traceback: parity (every family,
# fuzz), then throughput for K=5 and the forced K=7 / K=9 generic path.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
o=gpurun_out/r02lds; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
: > $o/bench.txt
for args in "--K 5" "--K 5 --hard" "--K 7" "--K 9 --hard"; do
  VTB_KERNEL=lds timeout -k 10 200 python3 bench.py $args --steps 20 --warmup 3 --cpu-seconds 0 > $o/b.json 2> $o/b.err || exit $?
  echo "lds $args $(python3 -c "import json;d=json.load(open('$o/b.json'));print(d['value'], d['roofline']['kernel_ms'])")" >> $o/bench.txt
done
cat $o/bench.txt
exit 0
