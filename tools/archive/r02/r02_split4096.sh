#!/bin/bash
# A/B on one box: the 4,096 x 1,024 soft headline with the default kernel (two frames per
# wave, 2 waves per SIMD) against the persistent split kernel (VTB_KERNEL=k7s: one frame per
# wave as two halves), warm-up 48 / 96; three interleaved rounds; then hard input.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
o=gpurun_out/r02split; mkdir -p $o
run() {  # tag env... -- bench args
  local tag=$1; shift
  env "$@" timeout -k 10 120 python3 bench.py --steps 50 --warmup 5 --cpu-seconds 0 $BARGS > $o/$tag.json 2> $o/$tag.err || { tail -5 $o/$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$o/$tag.json')); print('$tag', round(d['value']), d['ms_per_step'], d['roofline'].get('per_launch_pass_ms'))"
}
for r in 1 2 3; do
  BARGS=""; run soft_default_$r VTB_X=0; run soft_k7s_w48_$r VTB_KERNEL=k7s VTB_SPLIT_WARM=48; run soft_k7s_w96_$r VTB_KERNEL=k7s VTB_SPLIT_WARM=96
done
for r in 1 2; do
  BARGS="--hard"; run hard_default_$r VTB_X=0; run hard_k7s_w48_$r VTB_KERNEL=k7s VTB_SPLIT_WARM=48
done
BARGS="--frames 8192"; run soft8k_default VTB_X=0; run soft8k_k7s_w48 VTB_KERNEL=k7s VTB_SPLIT_WARM=48
exit 0
