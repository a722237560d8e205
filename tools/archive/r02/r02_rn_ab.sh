#!/bin/bash
# Soft renormalisation period A/B (VTB_EXP_RN, tools/build_variants.sh base rn16): the full GPU
# suite on the rn16 build, then interleaved bench rounds of both builds on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
VTB_LIB_PATH=$PWD/convolutionalencdec_amd/lib/exp/rn16/libviterbi_amd.so timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/rn16_suite.log 2>&1 || { tail -30 gpurun_out/rn16_suite.log; exit 1; }
tail -1 gpurun_out/rn16_suite.log
bash tools/ab_variants.sh 6 > gpurun_out/ab_rn_soft.txt || exit 1
cat gpurun_out/ab_rn_soft.txt
bash tools/ab_variants.sh 3 --frames 65536 --frame-bits 2048 --gen device > gpurun_out/ab_rn_c3.txt || exit 1
cat gpurun_out/ab_rn_c3.txt
