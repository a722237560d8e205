#!/bin/bash
# Rehearsal of bench.py's N > 1 path on a one-GPU box: N ranks under torchrun, all on device 0,
# gloo for the barrier and the max-over-ranks (the driver's 8-GPU run uses RCCL, one GPU each).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05
n=${1:-2}
VTB_BENCH_ONE_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus $n --steps 10 --warmup 3 --dist-backend gloo \
  > gpurun_out/r05/dist_rehearsal_${n}ranks_one_gpu.json 2> gpurun_out/r05/dist_rehearsal_$n.err || { tail -20 gpurun_out/r05/dist_rehearsal_$n.err; exit 1; }
cat gpurun_out/r05/dist_rehearsal_${n}ranks_one_gpu.json
