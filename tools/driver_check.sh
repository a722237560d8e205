#!/bin/bash
# The driver's round-end GPU steps on this tree: pytest -m gpu, smoke(), the bench command.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/${ROUND:-r06}
timeout -k 10 600 python -m pytest tests/ -x -q -m gpu -p no:cacheprovider > gpurun_out/${ROUND:-r06}/driver_gputests.log 2>&1 || { tail -30 gpurun_out/${ROUND:-r06}/driver_gputests.log; exit 1; }
tail -2 gpurun_out/${ROUND:-r06}/driver_gputests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${ROUND:-r06}/driver_smoke.log 2>&1 || { cat gpurun_out/${ROUND:-r06}/driver_smoke.log; exit 1; }
tail -1 gpurun_out/${ROUND:-r06}/driver_smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${ROUND:-r06}/driver_bench.json 2> gpurun_out/${ROUND:-r06}/driver_bench.err || exit 1
cut -c1-330 gpurun_out/${ROUND:-r06}/driver_bench.json
