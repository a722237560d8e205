#!/bin/bash
# Launch time vs batch size for the K=7 soft workload (measurement only).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/fscan.txt
: > $out
for kern in "" gws; do
for F in 2048 4096 6144 8192 10240 12288 16384 32768 65536; do
  r=$(VTB_KERNEL=$kern timeout -k 10 120 python bench.py --steps 50 --warmup 5 --cpu-seconds 0 --frames $F 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['roofline']['kernel_ms']*1000,2), round(d['value']/1000,1))") || exit 1
  echo "kernel=${kern:-auto} F=$F kernel_us,Gbps=$r" | tee -a $out
done
done
