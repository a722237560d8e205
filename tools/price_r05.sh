#!/bin/bash
# Round 5 pricing runs, each under its own limit:
#   acs2   tools/probes/acs2_probe (two-register layout with the real loop's overhead; the
#          4,096 x 1,024 soft launch fed with split halves)
#   k9     K=9 hard at 2 waves per SIMD (4,096 x 1,024) against 4 (8,192 half-length frames:
#          what splitting every K=9 frame in two would run), three interleaved rounds
#   k9sq   SQ counter passes of both K=9 shapes (where the wave cycles go)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05
mkdir -p $O
for step in "$@"; do
  case $step in
    acs2)
      timeout -k 10 120 tools/probes/acs2_probe > $O/acs2_probe.txt 2>&1 || { cat $O/acs2_probe.txt; exit 1; }
      cat $O/acs2_probe.txt ;;
    k9)
      : > $O/k9_waves_ab.jsonl
      for r in 1 2 3; do
        for fb in 1024 512 520 496; do
          fr=$(( fb == 1024 ? 4096 : 8192 ))
          timeout -k 10 120 python bench.py --K 9 --hard --frames $fr --frame-bits $fb --steps 100 --warmup 5 --cpu-seconds 0 \
            > $O/k9_tmp.json 2> $O/k9_tmp.err || { tail $O/k9_tmp.err; exit 1; }
          python3 -c "import json,sys; d=json.load(open('$O/k9_tmp.json')); r=d['roofline']; print(json.dumps({'round': $r, 'frames': $fr, 'frame_bits': $fb, 'value': d['value'], 'kernel_avg_ms': r['kernel_avg_ms'], 'ms_per_step': d['ms_per_step']}))" | tee -a $O/k9_waves_ab.jsonl
        done
      done ;;
    k9sq)
      # SQ wave-cycle passes (tools/pmc_stalls.sh) of both K=9 shapes
      TAG=c4 BARGS="--K 9 --hard" timeout -k 10 400 bash tools/pmc_stalls.sh || exit 1
      TAG=c4x4 BARGS="--K 9 --hard --frames 8192 --frame-bits 512" timeout -k 10 400 bash tools/pmc_stalls.sh || exit 1
      python3 tools/stalls_summary.py gpurun_out/stalls_c4 $O/sq_c4_4096x1024.json "K9 hard 4096 x 1024, 2 waves/SIMD"
      python3 tools/stalls_summary.py gpurun_out/stalls_c4x4 $O/sq_c4_8192x512.json "K9 hard 8192 x 512, 4 waves/SIMD" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
