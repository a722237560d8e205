#!/bin/bash
# Fixed per-launch cost of the K=7 kernel (measurement only): HIP-event launch time with
# VTB_DEBUG = 16 (return at entry), 3 (first chunk staged, no ACS / traceback), 0 (full),
# at several batch sizes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/breakdown2.txt
: > $out
for F in 256 1024 4096 8192; do
  for d in 16 3 1 0; do
    r=$(VTB_DEBUG=$d timeout -k 10 120 python bench.py --steps 50 --warmup 5 --cpu-seconds 0 --frames $F 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['roofline']['kernel_ms']*1000, d['ms_per_step']*1000)") || exit 1
    echo "F=$F dbg=$d kernel_us,step_us=$r" | tee -a $out
  done
done
