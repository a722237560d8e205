#!/bin/bash
# Every fuzz family of tests/test_gpu_fuzz.py (batch cases at listed and arbitrary lengths,
# single-frame path, streams, general-k, random generators, hard hybrid) at VTB_FUZZ_N cases per
# seed, seeds from the arguments; one summary line per seed.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/fuzzall; mkdir -p $o
export TMPDIR=/tmp
for seed in "$@"; do
  VTB_FUZZ_N=${VTB_FUZZ_N:-2000} VTB_FUZZ_SEED=$seed timeout -k 10 1000 python3 -u -m pytest tests/test_gpu_fuzz.py -q -p no:cacheprovider --timeout 300 --timeout-method thread > $o/seed$seed.log 2>&1
  rc=$?
  echo "seed $seed: exit $rc $(tail -1 $o/seed$seed.log)"
  grep "^FAILED" $o/seed$seed.log | head -10
  [ $rc -eq 0 ] || exit $rc
done
exit 0
