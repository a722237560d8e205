#!/bin/bash
# Round 2: reproduce the driver's bench command (--steps 20 --warmup 5) with per-launch
# events, next to longer runs, and a rocprofv3 kernel-trace of the driver-exact command.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out/r02gap
export TMPDIR=/tmp
o=gpurun_out/r02gap
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 > $o/drv1.json 2> $o/drv1.err || exit $?
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 > $o/drv2.json 2> $o/drv2.err || exit $?
timeout -k 10 200 python3 bench.py --gpus 1 --steps 200 --warmup 5 --cpu-seconds 0 > $o/s200.json 2> $o/s200.err || exit $?
rm -rf $o/prof
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 > $o/prof.json 2> $o/prof.err || exit $?
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $o/full.json 2> $o/full.err || exit $?
exit 0
