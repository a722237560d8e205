#!/bin/bash
# C3 ACS only (VTB_DEBUG=1): survivor-word stores (base) vs none (noword variant, wrong
# output), global-survivor kernel.  Measurement only.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/c3_store_ab.txt; : > $out
for r in 1 2; do
  for d in convolutionalencdec_amd/lib/exp/*/; do
    n=$(basename $d)
    v=$(VTB_LIB_PATH=$PWD/$d/libviterbi_amd.so VTB_DEBUG=1 timeout -k 10 120 python bench.py --steps 10 --warmup 2 --cpu-seconds 0 --frames 65536 --frame-bits 2048 --gen device 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['roofline']['kernel_ms']*1000,1))") || exit 1
    w=$(VTB_LIB_PATH=$PWD/$d/libviterbi_amd.so VTB_KERNEL=gws VTB_DEBUG=1 timeout -k 10 120 python bench.py --steps 20 --warmup 2 --cpu-seconds 0 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['roofline']['kernel_ms']*1000,2))") || exit 1
    echo "$n C3_acs_us=$v gws4096_acs_us=$w" | tee -a $out
  done
done
