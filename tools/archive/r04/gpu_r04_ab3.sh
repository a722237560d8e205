#!/bin/bash
# Round 4: price the K=9 permlane swaps (measurement build with plain moves, wrong results).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04
E=convolutionalencdec_amd/lib/exp
VARIANTS="$E/base $E/k9noswap" VTB_DEBUG=1 bash tools/ab_variants.sh 3 --K 9 --hard && cp gpurun_out/ab.txt gpurun_out/r04/ab_k9noswap_acs_only.txt
