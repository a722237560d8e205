#!/bin/bash
# Streaming decoder: this call's survivor words in LDS (default) vs the global ring only
# (VTB_DEBUG=64), per call length.  Measurement only.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/stream_ab.txt; : > $out
for r in 1 2; do
  for C in 480 1008 4080; do
    for d in 0 64; do
      v=$(VTB_DEBUG=$d timeout -k 10 120 python bench.py --steps 30 --warmup 3 --cpu-seconds 0 --stream-chunk $C $EXTRA 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step']*1000,2), round(d['value']/1000,1))") || exit 1
      echo "C=$C dbg=$d us_per_call,Gbps=$v" | tee -a $out
    done
  done
done
