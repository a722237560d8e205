#!/bin/bash
# A/B of libraries on one box: each of $AB_LIBS (space-separated paths to alternative builds of
# libviterbi_amd.so loaded through VTB_LIB_PATH; "shipped" = the in-tree library), interleaved
# rounds of bench.py runs (HIP-event kernel time of 100 back-to-back launches).  Measurement only.
#   usage: AB_LIBS="shipped convolutionalencdec_amd/lib/exp/<name>/libviterbi_amd.so" \
#          bash tools/ab_lib.sh OUT ROUNDS "cfg1" "cfg2" ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=$1; rounds=$2; shift 2
mkdir -p "$(dirname "$out")"
: > "$out"
for r in $(seq 1 "$rounds"); do
  for cfg in "$@"; do
    for lib in ${AB_LIBS:-shipped}; do
      if [ "$lib" = shipped ]; then unset VTB_LIB_PATH; else export VTB_LIB_PATH=$lib; fi
      timeout -k 10 120 python bench.py $cfg --steps 100 --warmup 5 --cpu-seconds 0 > "$out.tmp" 2> "$out.err" || { tail "$out.err"; exit 1; }
      python3 -c "import json; d=json.load(open('$out.tmp')); r=d['roofline']; print(json.dumps({'round': $r, 'cfg': '$cfg', 'lib': '$lib', 'kernel': r['secondary'].get('kernel'), 'value': d['value'], 'kernel_avg_ms': r['kernel_avg_ms']}))" | tee -a "$out"
    done
  done
done
unset VTB_LIB_PATH
rm -f "$out.tmp"
