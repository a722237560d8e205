#!/bin/bash
# Round-5 GPU steps, each under its own time limit, stopping at the first failure.
#   tools/gpu_r05.sh guard   the completeness-guard tests (tests/test_gpu_tb_guard.py)
#   tools/gpu_r05.sh suite   the whole GPU suite, smoke() and the driver's bench command
#   tools/gpu_r05.sh bench   the driver's bench command only (twice)
#   tools/gpu_r05.sh prof    rocprofv3 kernel trace + stats of the bench command
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05
mkdir -p $O
sha=$(sha256sum convolutionalencdec_amd/lib/libviterbi_amd.so | cut -c1-16)
echo "lib sha16 $sha" | tee $O/lib_sha16.txt
PYT="python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread"
for step in "$@"; do
  case $step in
    guard)
      timeout -k 10 600 ${PYT/-x /} tests/test_gpu_tb_guard.py -m gpu > $O/guard.log 2>&1 || { tail -40 $O/guard.log; exit 1; }
      tail -2 $O/guard.log ;;
    suite)
      timeout -k 10 900 $PYT tests/ -m gpu > $O/gpu_tests_full.log 2>&1 || { tail -40 $O/gpu_tests_full.log; exit 1; }
      tail -2 $O/gpu_tests_full.log
      timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
      tail -1 $O/smoke.log
      timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
      cut -c1-400 $O/bench.json ;;
    bench)
      for i in 1 2; do
        timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_$i.json 2> $O/bench_$i.err || { tail $O/bench_$i.err; exit 1; }
        cut -c1-300 $O/bench_$i.json
      done ;;
    prof)
      cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof_bench.json 2> $O/prof.err || { tail $O/prof.err; exit 1; }
      find $O/prof -name '*kernel_stats.csv' | head -3 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
