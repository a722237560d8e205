#!/bin/bash
# Round 4: priority share on C3 (persistent split kernel) and C2 (hard), base = 67 %.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04
E=convolutionalencdec_amd/lib/exp
V="$E/base $E/prio59 $E/prio75 $E/prio85"
VARIANTS="$V" bash tools/ab_variants.sh 3 --frames 65536 --frame-bits 2048 --gen device && cp gpurun_out/ab.txt gpurun_out/r04/ab_prio_c3.txt || exit 1
VARIANTS="$V" bash tools/ab_variants.sh 3 --hard && cp gpurun_out/ab.txt gpurun_out/r04/ab_prio_c2.txt || exit 1
# K=9 (C4): the K=7 wave balance added to the K=9 frame kernel (measurement builds)
VARIANTS="$E/base $E/k9prio59 $E/k9prio67 $E/k9prio75" bash tools/ab_variants.sh 3 --K 9 --hard && cp gpurun_out/ab.txt gpurun_out/r04/ab_prio_c4.txt
