#!/bin/bash
# Round 4: the second wave's priority share (kPrioPct) A/B on the headline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04
E=convolutionalencdec_amd/lib/exp
VARIANTS="$E/base $E/prio63 $E/prio67 $E/prio71" bash tools/ab_variants.sh 6 && cp gpurun_out/ab.txt gpurun_out/r04/ab_prio_2.txt
