#!/bin/bash
# Rehearsal of bench.py's N > 1 path on a one-GPU box: torchrun ranks all on device 0
# (VTB_BENCH_ONE_DEVICE=1), barrier and max-reduction over gloo (RCCL refuses two ranks on one
# GPU).  Checks the launcher, per-rank shards, Timer and rank-0 JSON; the ranks share one GPU,
# so the value is not a scaling number.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
o=gpurun_out/r02dist; mkdir -p $o
export VTB_BENCH_ONE_DEVICE=1
for n in 2 4; do
  timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29500 + n)) bench.py --gpus $n --steps 20 --warmup 5 --dist-backend gloo > $o/n$n.json 2> $o/n$n.err \
    || { tail -20 $o/n$n.err; exit 1; }
  python3 -c "import json; ls=[l for l in open('$o/n$n.json') if l.startswith('{')]; assert len(ls)==1, ls; d=json.loads(ls[0]); print($n, d['n_gpus'], round(d['value']), d['ms_per_step'], d['config']['global_batch_frames'], d['cpu_baseline'])"
done
exit 0
