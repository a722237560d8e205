#!/bin/bash
# Round 4: SQ stall / LDS passes (headline with and without the traceback, C4) and the K=9
# non-temporal survivor-store A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
E=convolutionalencdec_amd/lib/exp
VARIANTS="$E/base $E/k9nt" bash tools/ab_variants.sh 3 --K 9 --hard && cp gpurun_out/ab.txt gpurun_out/r04/ab_k9nt.txt || exit 1
TAG=head bash tools/pmc_stalls.sh || exit 1
TAG=notb VTB_DEBUG=1 bash tools/pmc_stalls.sh || exit 1
TAG=c4 BARGS="--K 9 --hard" bash tools/pmc_stalls.sh || exit 1
bash tools/configs.sh && cp gpurun_out/configs.jsonl gpurun_out/r04/configs.jsonl || exit 1
echo "ab2 done"
