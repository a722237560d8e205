#!/bin/bash
# A/B on one box: persistent grid (VTB_DEBUG=0) vs one wave per frame pair (VTB_DEBUG=32),
# LDS and global-survivor K=7 variants, soft, by batch size.  Measurement only.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/fscan_ab.txt
: > $out
for F in ${FLIST:-4096 8192 12288 16384 65536}; do
  for kern in k7 gws; do
    for d in 0 32 0 32; do
      r=$(VTB_KERNEL=$kern VTB_DEBUG=$d timeout -k 10 120 python bench.py --steps 50 --warmup 5 --cpu-seconds 0 --frames $F $EXTRA 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['roofline']['kernel_ms']*1000,2))") || exit 1
      echo "F=$F kernel=$kern dbg=$d kernel_us=$r" | tee -a $out
    done
  done
done
