#!/bin/bash
# Round 2: the streaming fuzz family (tests/test_gpu_fuzz.py test_stream_random_chunking_vs_oracle)
# at its default size and at VTB_FUZZ_N / 8 cases per seed.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
o=gpurun_out/streamfuzz; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fuzz.py -k stream -q -p no:cacheprovider --timeout 200 --timeout-method thread > $o/default.log 2>&1 || { tail -40 $o/default.log; exit 1; }
tail -1 $o/default.log
for seed in ${@:-31337 2026}; do
  VTB_FUZZ_N=${VTB_FUZZ_N:-1600} VTB_FUZZ_SEED=$seed timeout -k 10 900 python3 -u -m pytest tests/test_gpu_fuzz.py -k stream -q -p no:cacheprovider --timeout 300 --timeout-method thread > $o/seed$seed.log 2>&1 || { tail -40 $o/seed$seed.log; exit 1; }
  tail -1 $o/seed$seed.log
done
exit 0
