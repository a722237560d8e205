#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
VTB_LIB_PATH=$PWD/convolutionalencdec_amd/lib/exp/swz/libviterbi_amd.so timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/swz_suite.log 2>&1 || { tail -30 gpurun_out/swz_suite.log; exit 1; }
tail -1 gpurun_out/swz_suite.log
bash tools/ab_variants.sh 4 > gpurun_out/ab_soft.txt || exit 1
cat gpurun_out/ab_soft.txt
bash tools/ab_variants.sh 3 --hard > gpurun_out/ab_hard.txt || exit 1
cat gpurun_out/ab_hard.txt
