#!/bin/bash
# Round 2: single-call latency probe (tools/probes/latency_probe.hip), the driver's bench
# command twice, and the reference speedDecode harness against the legacy drop-in.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
o=gpurun_out/r02lat; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 60 tools/probes/latency_probe > $o/latency_probe.txt 2>&1 || exit $?
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 > $o/drv1.json 2> $o/drv1.err || exit $?
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 > $o/drv2.json 2> $o/drv2.err || exit $?
timeout -k 10 60 bash tools/speed_decode.sh 5 > $o/speed_decode.txt 2>&1 || exit $?
exit 0
