#!/bin/bash
# GPU steps of a round (output under gpurun_out/$ROUND, default r06), each under its own time
# limit, stopping at the first failure.
#   tools/gpu_round.sh guard   the completeness-guard tests (tests/test_gpu_tb_guard.py)
#   tools/gpu_round.sh suite   the whole GPU suite, smoke() and the driver's bench command
#   tools/gpu_round.sh bench   the driver's bench command only (twice)
#   tools/gpu_round.sh prof    rocprofv3 kernel trace + stats of the bench command (the library's
#                            sha beside it for tools/kernel_time_summary.py)
#   tools/gpu_round.sh fuzz    one fuzz sweep and one fix-up sweep on this library (2,000 cases per
#                            family), plus the fuzz sweep again with every traceback verification
#                            forced to the guards' slow paths (VTB_DEBUG bit 17)
#   tools/gpu_round.sh stamps  PMC passes of every config line, the config lines, SQ passes of the
#                            headline (summarised on the CPU: tools/traffic_summary.py, ...)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${ROUND:-r06}
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
      export TMPDIR=/tmp
      rm -rf $O/prof && mkdir -p $O/prof && echo "$sha" > $O/prof/lib_sha16.txt
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof_bench.json 2> $O/prof.err || { tail $O/prof.err; exit 1; }
      find $O/prof -name '*kernel_stats.csv' | head -3 ;;
    fuzz)
      mkdir -p $O/fuzz
      VTB_FUZZ_N=2000 VTB_FUZZ_SEED=${FUZZ_SEED:-6005} timeout -k 10 900 ${PYT/-x /} tests/test_gpu_fuzz.py -m gpu > $O/fuzz/fuzz_seed${FUZZ_SEED:-6005}.log 2>&1 || { tail -30 $O/fuzz/fuzz_seed${FUZZ_SEED:-6005}.log; exit 1; }
      tail -n 1 $O/fuzz/fuzz_seed${FUZZ_SEED:-6005}.log
      VTB_FIXUP_N=2000 VTB_FIXUP_SEED=${FIXUP_SEED:-6007} timeout -k 10 600 ${PYT/-x /} tests/test_gpu_split_fixup.py -m gpu -k fixup_family > $O/fuzz/fixup_seed${FIXUP_SEED:-6007}.log 2>&1 || { tail -30 $O/fuzz/fixup_seed${FIXUP_SEED:-6007}.log; exit 1; }
      tail -n 1 $O/fuzz/fixup_seed${FIXUP_SEED:-6007}.log
      VTB_DEBUG=131072 VTB_FUZZ_N=2000 VTB_FUZZ_SEED=${FORCED_SEED:-6006} timeout -k 10 900 ${PYT/-x /} tests/test_gpu_fuzz.py -m gpu > $O/fuzz/fuzz_forced_seed${FORCED_SEED:-6006}.log 2>&1 || { tail -30 $O/fuzz/fuzz_forced_seed${FORCED_SEED:-6006}.log; exit 1; }
      tail -n 1 $O/fuzz/fuzz_forced_seed${FORCED_SEED:-6006}.log ;;
    stamps)
      timeout -k 10 900 bash tools/pmc_passes.sh head c2 c3s c3h c4 c5 || exit 1
      timeout -k 10 600 bash tools/configs.sh && cp gpurun_out/configs.jsonl $O/configs.jsonl || exit 1
      TAG=head timeout -k 10 400 bash tools/pmc_stalls.sh || exit 1 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
