#!/bin/bash
# Round 2: the persistent split kernel's next-frame prefetch as compiler-visible loads.  The
# failing fuzz cases replayed (bad frames and the split list count must be the same run to run),
# the full GPU suite, three 2,000-case fuzz sweeps, C3 throughput.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
o=gpurun_out/prefetchfix; mkdir -p $o
export TMPDIR=/tmp
VTB_FUZZ_N=2000 VTB_FUZZ_SEED=31337 timeout -k 10 300 python3 tools/dbg_batch_case.py 1173 1833 > $o/batch.jsonl 2> $o/batch.err || exit 1
cut -c1-260 $o/batch.jsonl
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $o/gpu_tests.log 2>&1 || { tail -30 $o/gpu_tests.log; exit 1; }
tail -1 $o/gpu_tests.log
VTB_FUZZ_N=2000 timeout -k 10 900 bash tools/r02_fuzz_long.sh 31337 424242 7 || exit 1
timeout -k 10 120 python3 bench.py --frames 65536 --frame-bits 2048 --gen device --steps 10 --warmup 2 --cpu-seconds 0 > $o/c3.json 2> $o/c3.err || exit 1
cut -c1-200 $o/c3.json
exit 0
