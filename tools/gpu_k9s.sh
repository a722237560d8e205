#!/bin/bash
# K=9 one-frame-per-wave kernel bring-up, each step under its own limit:
#   check  tools/k9s_check.py (oracle parity, shipped / forced guards / pair kernel)
#   ab     C4 (4,096 x 1,024 hard) and K=9 soft, k9s against the pair kernel (VTB_DEBUG bit 18),
#          three interleaved rounds of 100 back-to-back launches
#   occ    the crossover batch sizes (1,024 to 8,192 frames), two rounds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05/k9s
mkdir -p $O
for step in "$@"; do
  case $step in
    check)
      timeout -k 10 300 python -u tools/k9s_check.py > $O/check.log 2>&1 || { tail -40 $O/check.log; exit 1; }
      tail -3 $O/check.log ;;
    ab)
      : > $O/ab.jsonl
      for r in 1 2 3; do
        for cfg in "--hard" "" "--hard --frames 65536" "--frames 16384"; do
          for dbg in 0 262144; do
            VTB_DEBUG=$dbg timeout -k 10 120 python bench.py --K 9 $cfg --steps 100 --warmup 5 --cpu-seconds 0 \
              > $O/tmp.json 2> $O/tmp.err || { tail $O/tmp.err; exit 1; }
            python3 -c "import json; d=json.load(open('$O/tmp.json')); r=d['roofline']; print(json.dumps({'round': $r, 'cfg': '$cfg', 'dbg': $dbg, 'kernel': r['secondary'].get('kernel'), 'value': d['value'], 'kernel_avg_ms': r['kernel_avg_ms']}))" | tee -a $O/ab.jsonl
          done
        done
      done ;;
    occ)
      # the k9s / pair crossover: batches from 1,024 to 8,192 frames (up to one k9s round), two rounds
      : > $O/occ.jsonl
      for r in 1 2; do
        for cfg in "--frames 1024" "--hard --frames 2048" "--frames 6144" "--hard --frames 6144" "--frames 8192" "--hard --frames 8192"; do
          for dbg in 0 262144; do
            VTB_DEBUG=$dbg timeout -k 10 120 python bench.py --K 9 $cfg --steps 100 --warmup 5 --cpu-seconds 0 \
              > $O/tmp.json 2> $O/tmp.err || { tail $O/tmp.err; exit 1; }
            python3 -c "import json; d=json.load(open('$O/tmp.json')); r=d['roofline']; print(json.dumps({'round': $r, 'cfg': '$cfg', 'dbg': $dbg, 'kernel': r['secondary'].get('kernel'), 'value': d['value'], 'kernel_avg_ms': r['kernel_avg_ms']}))" | tee -a $O/occ.jsonl
          done
        done
      done ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
