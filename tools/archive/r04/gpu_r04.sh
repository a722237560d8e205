#!/bin/bash
# Round 4 GPU steps, each under its own time limit, stopping at the first failure:
#   bash tools/gpu_r04.sh tests:<pytest args> | gputests | smoke | bench | bench50 | prof | fixup2000 | seed1017 ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/r04; mkdir -p $o
export TMPDIR=/tmp
for s in "$@"; do
  case $s in
    tests:*) t="${s#tests:}"; n=$(echo "$t" | tr -c 'a-zA-Z0-9_' '_' | cut -c1-60)
             timeout -k 10 900 python3 -u -m pytest $t -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
               > $o/tests_$n.log 2>&1 || { tail -40 $o/tests_$n.log; exit 1; } ; tail -3 $o/tests_$n.log ;;
    gputests) timeout -k 10 1100 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
               > $o/gpu_tests_full.log 2>&1 || { tail -40 $o/gpu_tests_full.log; exit 1; } ; tail -3 $o/gpu_tests_full.log ;;
    fixup2000) VTB_FIXUP_N=2000 VTB_FIXUP_SEED=424242 timeout -k 10 1100 python3 -u -m pytest tests/test_gpu_split_fixup.py -q \
               -p no:cacheprovider --timeout 300 --timeout-method thread -k fixup_family > $o/fixup_sweep_2000.log 2>&1 \
               || { tail -40 $o/fixup_sweep_2000.log; exit 1; } ; tail -3 $o/fixup_sweep_2000.log ;;
    seed1017) VTB_FUZZ_N=2000 VTB_FUZZ_SEED=1017 timeout -k 10 1100 python3 -u -m pytest tests/test_gpu_fuzz.py -q \
               -p no:cacheprovider --timeout 300 --timeout-method thread > $o/fuzz_seed1017.log 2>&1 \
               || { tail -40 $o/fuzz_seed1017.log; exit 1; } ; tail -3 $o/fuzz_seed1017.log ;;
    fuzz:*) sd="${s#fuzz:}"; VTB_FUZZ_N=${FUZZ_N:-2000} VTB_FUZZ_SEED=$sd timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fuzz.py -q \
               -p no:cacheprovider --timeout 300 --timeout-method thread > $o/fuzz_seed$sd.log 2>&1 \
               || { tail -40 $o/fuzz_seed$sd.log; exit 1; } ; tail -2 $o/fuzz_seed$sd.log ;;
    fixup:*) sd="${s#fixup:}"; VTB_FIXUP_N=${FIXUP_N:-2000} VTB_FIXUP_SEED=$sd timeout -k 10 600 python3 -u -m pytest tests/test_gpu_split_fixup.py -q \
               -p no:cacheprovider --timeout 300 --timeout-method thread -k fixup_family > $o/fixup_seed$sd.log 2>&1 \
               || { tail -40 $o/fixup_seed$sd.log; exit 1; } ; tail -2 $o/fixup_seed$sd.log ;;
    smoke) timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { cat $o/smoke.log; exit 1; } ;;
    bench) timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $o/bench.json 2> $o/bench.err || { tail $o/bench.err; exit 1; }
           cat $o/bench.json ;;
    bench50) timeout -k 10 300 python3 bench.py --gpus 1 --steps 50 --warmup 5 --cpu-seconds 0 > $o/bench50.json 2> $o/bench50.err || exit 1
           cat $o/bench50.json ;;
    prof) rm -rf $o/prof
          timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 > $o/prof.json 2> $o/prof.err || { tail $o/prof.err; exit 1; } ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
exit 0
