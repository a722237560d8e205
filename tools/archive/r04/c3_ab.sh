#!/bin/bash
# A/B of the prebuilt variant libraries on config C3 (65,536 x 2,048-bit soft frames,
# device-generated), interleaved.  Measurement only.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/c3_ab.txt; : > $out
for r in 1 2 3; do
  for d in convolutionalencdec_amd/lib/exp/*/; do
    n=$(basename $d)
    v=$(VTB_LIB_PATH=$PWD/$d/libviterbi_amd.so timeout -k 10 120 python bench.py --steps 10 --warmup 2 --cpu-seconds 0 --frames 65536 --frame-bits 2048 --gen device "$@" 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['roofline']['kernel_ms']*1000,1), round(d['value']/1000,1))") || exit 1
    echo "$n kernel_us,Gbps=$v" | tee -a $out
  done
done
