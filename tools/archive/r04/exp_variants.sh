#!/bin/bash
# Time each prebuilt variant library (convolutionalencdec_amd/lib/exp/*) with bench.py, whole
# kernel and ACS only (VTB_DEBUG=1 skips the traceback).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for d in convolutionalencdec_amd/lib/exp/*/; do
  n=$(basename $d)
  VTB_LIB_PATH=$PWD/$d/libviterbi_amd.so timeout -k 10 120 python bench.py --steps 30 --warmup 3 --cpu-seconds 0 > gpurun_out/var_$n.log 2>&1 || exit $?
  VTB_DEBUG=1 VTB_LIB_PATH=$PWD/$d/libviterbi_amd.so timeout -k 10 120 python bench.py --steps 30 --warmup 3 --cpu-seconds 0 > gpurun_out/var_${n}_acsonly.log 2>&1 || exit $?
  VTB_DEBUG=1 VTB_LIB_PATH=$PWD/$d/libviterbi_amd.so timeout -k 10 120 python bench.py --steps 30 --warmup 3 --cpu-seconds 0 --frames 2048 > gpurun_out/var_${n}_acsonly_1w.log 2>&1 || exit $?
done
