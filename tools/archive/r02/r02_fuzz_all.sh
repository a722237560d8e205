#!/bin/bash
# Round 2: every fuzz family of tests/test_gpu_fuzz.py at VTB_FUZZ_N per seed (seeds from the
# arguments).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
o=gpurun_out/fuzzall; mkdir -p $o
export TMPDIR=/tmp
for seed in "$@"; do
  VTB_FUZZ_N=${VTB_FUZZ_N:-2000} VTB_FUZZ_SEED=$seed timeout -k 10 1000 python3 -u -m pytest tests/test_gpu_fuzz.py -q -p no:cacheprovider --timeout 300 --timeout-method thread > $o/seed$seed.log 2>&1
  echo "seed $seed: exit $? $(tail -1 $o/seed$seed.log)"
  grep "^FAILED" $o/seed$seed.log | head -10
done
exit 0
