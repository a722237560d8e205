#!/bin/bash
# Split frames (one frame per wave, both halves at once) vs the normal two-frame waves
# (VTB_DEBUG=256), small batches, soft and hard.  Measurement only.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/split_ab.txt; : > $out
for wl in "" "--hard"; do
  for cfg in "--frames 1 --frame-bits 2048" "--frames 256 --frame-bits 1024" "--frames 1024 --frame-bits 1024" "--frames 2048 --frame-bits 1024" "--frames 2048 --frame-bits 2048"; do
    for d in 0 256; do
      v=$(VTB_DEBUG=$d timeout -k 10 120 python bench.py --steps 50 --warmup 5 --cpu-seconds 0 $cfg $wl 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['roofline']['kernel_ms']*1000,2), round(d['value']/1000,2), d['config']['decoded_ber'])") || exit 1
      echo "$cfg $wl dbg=$d kernel_us,Gbps,ber=$v" | tee -a $out
    done
  done
done
