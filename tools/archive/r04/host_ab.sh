#!/bin/bash
# PCIe-inclusive host-path rate (bench.py config.host_buffers_mbps) of the prebuilt variant
# libraries (convolutionalencdec_amd/lib/exp/*), interleaved.  Measurement only.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/host_ab.txt; : > $out
for r in 1 2; do
  for F in 4096 65536; do
    for d in convolutionalencdec_amd/lib/exp/*/; do
      n=$(basename $d)
      v=$(VTB_LIB_PATH=$PWD/$d/libviterbi_amd.so timeout -k 10 120 python bench.py --steps 5 --warmup 2 --cpu-seconds 0 --frames $F 2>/dev/null | grep -o '"host_buffers_mbps": [0-9.]*' | cut -d' ' -f2) || exit 1
      echo "$n F=$F host_mbps=$v" | tee -a $out
    done
  done
done
