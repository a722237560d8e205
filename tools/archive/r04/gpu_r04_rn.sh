#!/bin/bash
# Round 4: soft renormalisation period 16 vs 12 on the final library (headline and C3).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04
E=convolutionalencdec_amd/lib/exp
VARIANTS="$E/base $E/rn16" bash tools/ab_variants.sh 6 && cp gpurun_out/ab.txt gpurun_out/r04/ab_rn16.txt || exit 1
VARIANTS="$E/base $E/rn16" bash tools/ab_variants.sh 3 --frames 65536 --frame-bits 2048 --gen device && cp gpurun_out/ab.txt gpurun_out/r04/ab_rn16_c3.txt
