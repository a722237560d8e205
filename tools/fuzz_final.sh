#!/bin/bash
# The per-library fuzz sweeps (tools/gpu_round.sh fuzz) plus the widened stream sweep (2,000 stream
# cases of every K), output under gpurun_out/$ROUND/fuzz.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${ROUND:-r06}
bash tools/gpu_round.sh fuzz || exit 1
VTB_FUZZ_N=16000 VTB_FUZZ_SEED=6605 timeout -k 10 600 python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    tests/test_gpu_fuzz.py -m gpu -k stream_random > $O/fuzz/fuzz_stream_seed6605.log 2>&1 || { tail -30 $O/fuzz/fuzz_stream_seed6605.log; exit 1; }
tail -n 1 $O/fuzz/fuzz_stream_seed6605.log
