#!/bin/bash
# Phase breakdown from bench.py's HIP-event launch time: VTB_DEBUG = 0 (full), 1 (no
# traceback), 3 (neither ACS nor traceback: prologue/epilogue), 5 (traceback without
# verification rounds) for the K=7 and K=9 workloads.  Measurement only.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/breakdown.txt
: > $out
for wl in "--K 7" "--K 7 --hard" "--K 9 --hard" "--K 9"; do
  for d in 0 1 3 4; do
    r=$(VTB_DEBUG=$d timeout -k 10 120 python bench.py --steps 50 --warmup 5 --cpu-seconds 0 $wl $EXTRA 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['roofline']['kernel_ms']*1000)") || exit 1
    echo "$wl dbg=$d kernel_us=$r" | tee -a $out
  done
done
