#!/bin/bash
# Round 4 counter passes on the shipped library (summarise on the CPU afterwards):
#   PMC traffic + VALU for every config line (tools/pmc_r04.sh -> tools/traffic_summary.py r04),
#   SQ stall / LDS passes of the headline with and without the traceback (VTB_DEBUG=1), and C4.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/pmc_r04.sh ${WL:-head c2 c3s c3h c4 c5} || exit 1
echo "prof passes done"
