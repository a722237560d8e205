#!/bin/bash
# A/B on one box for the K=9 kernel: persistent grid (VTB_DEBUG=0) vs one wave per pair
# (VTB_DEBUG=32), hard and soft, by batch size.  Measurement only.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/fscan_k9.txt
: > $out
for F in 4096 8192 16384; do
  for wl in "--hard" ""; do
    for d in 0 32 0 32; do
      r=$(VTB_DEBUG=$d timeout -k 10 120 python bench.py --K 9 --steps 30 --warmup 3 --cpu-seconds 0 --frames $F $wl 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['roofline']['kernel_ms']*1000,2))") || exit 1
      echo "F=$F K9 $wl dbg=$d kernel_us=$r" | tee -a $out
    done
  done
done
