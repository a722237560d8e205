#!/bin/bash
# Round 2 checkpoint: full GPU suite, every BASELINE config (tools/configs.sh), the PMC passes
# of the shipped library (tools/r02_pmc.sh), the driver's bench command under rocprofv3.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r02final
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/r02final/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r02final/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r02final/gpu_tests.log
bash tools/configs.sh > gpurun_out/r02final/configs.txt 2>&1 || exit 1
cp gpurun_out/configs.jsonl gpurun_out/r02final/configs.jsonl
bash tools/r02_pmc.sh || exit 1
bash tools/r02_check.sh bench prof || exit 1
exit 0
