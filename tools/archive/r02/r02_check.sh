#!/bin/bash
# Round 2 GPU check: parity suite, smoke, the driver's bench command, timestamps, and the
# rocprofv3 kernel-trace summary of the driver's bench command.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
o=gpurun_out/r02check; mkdir -p $o
export TMPDIR=/tmp
what="${*:-tests smoke bench prof}"
for s in $what; do
  case $s in
    tests) timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $o/gpu_tests.log 2>&1 || { tail -30 $o/gpu_tests.log; exit 1; } ;;
    smoke) timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit $? ;;
    bench) timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $o/bench.json 2> $o/bench.err || exit $?
           timeout -k 10 120 python3 tools/tstamp.py > $o/tstamp.json 2> $o/tstamp.err || exit $? ;;
    prof) rm -rf $o/prof
          timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 > $o/prof.json 2> $o/prof.err || exit $? ;;
  esac
done
exit 0
