#!/bin/bash
# Every BASELINE.json configuration on one GPU box, one bench.py line each
# (profiles/<round>/configs.jsonl).  C1 is the reference's CPU path (cpu_baseline of the C2
# line); C5 runs its per-GPU share (2^20 / 8 = 131,072 frames) on one GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/configs.jsonl; : > $out
run() {  # label, bench args
  local label=$1; shift
  timeout -k 10 300 python bench.py "$@" 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); d['config']['baseline_config']='$label'; print(json.dumps(d))" >> $out || exit 1
  tail -1 $out | cut -c1-160
}
run C2 --hard --steps 50 --warmup 5 --cpu-seconds 5
run C3 --frames 65536 --frame-bits 2048 --gen device --steps 10 --warmup 2 --cpu-seconds 0
run C3-hard --frames 65536 --frame-bits 2048 --gen device --hard --steps 10 --warmup 2 --cpu-seconds 0
run C4 --K 9 --hard --steps 30 --warmup 3 --cpu-seconds 0
run C5-per-GPU --frames 131072 --gen device --steps 10 --warmup 2 --cpu-seconds 0
run headline --steps 50 --warmup 5 --cpu-seconds 0
