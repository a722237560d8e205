#!/bin/bash
# A longer seeded fuzz sweep (VTB_FUZZ_N cases per family, default 500; seeds from the
# arguments, default 777 4242) on the GPU box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
o=gpurun_out/r02fuzzlong; mkdir -p $o
export TMPDIR=/tmp
n=${VTB_FUZZ_N:-500}
for seed in ${@:-777 4242}; do
  VTB_FUZZ_N=$n VTB_FUZZ_SEED=$seed timeout -k 10 900 python3 -u -m pytest tests/test_gpu_fuzz.py -k "random_case or single_frame" -q -p no:cacheprovider --timeout 300 --timeout-method thread > $o/seed$seed.log 2>&1 || { tail -40 $o/seed$seed.log; exit 1; }
  tail -1 $o/seed$seed.log
done
exit 0
