#!/bin/bash
# A/B of the rate-1/3 kernels: tools/k1n_scan.py on a saved library (convolutionalencdec_amd/lib/exp/<name>)
# against the in-tree one, interleaved.  Usage (GPU box): bash tools/k1n_ab.sh <reps> <name>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/k1n_ab.txt; : > $out
for r in $(seq $1); do
  echo "## base ($2)" >> $out
  VTB_LIB_PATH=$PWD/convolutionalencdec_amd/lib/exp/$2/libviterbi_amd.so timeout -k 10 200 python3 tools/k1n_scan.py 2>/dev/null >> $out || exit 1
  echo "## in-tree" >> $out
  timeout -k 10 200 python3 tools/k1n_scan.py 2>/dev/null >> $out || exit 1
done
cat $out
