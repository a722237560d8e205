#!/bin/bash
# Round 4, the shipped library: full GPU suite, smoke, the driver's bench command, its
# rocprofv3 kernel stats, the PMC passes of every config line and the config lines themselves.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_r04.sh gputests smoke bench prof || exit 1
bash tools/pmc_r04.sh head c2 c3s c3h c4 c5 || exit 1
bash tools/configs.sh && cp gpurun_out/configs.jsonl gpurun_out/r04/configs.jsonl || exit 1
TAG=head bash tools/pmc_stalls.sh || exit 1
echo "final done"
