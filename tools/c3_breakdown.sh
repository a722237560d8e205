#!/bin/bash
# Config C3 (65,536 x 2,048-bit soft frames): launch time with and without the traceback
# (VTB_DEBUG=1), auto kernel choice and each K=7 variant.  Measurement only.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/c3_breakdown.txt; : > $out
for kern in "" gws k7; do
  for d in 0 1; do
    v=$(VTB_KERNEL=$kern VTB_DEBUG=$d timeout -k 10 120 python bench.py --steps 10 --warmup 2 --cpu-seconds 0 --frames 65536 --frame-bits 2048 --gen device 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['roofline']['kernel_ms']*1000,1), round(d['value']/1000,1))") || exit 1
    echo "kernel=${kern:-auto} dbg=$d kernel_us,Gbps=$v" | tee -a $out
  done
done
