"""The multi-GPU bench harness on CPU: two ranks over gloo (127.0.0.1), the same Timer,
barrier and max-over-ranks reduction bench.py uses over RCCL, and the per-rank shard
generation (frames are sharded with no data-path collective, SURVEY.md 8 e)."""
import os
import socket
import sys

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import time

    import bench
    from convolutionalencdec_amd import synth

    dist.init_process_group("gloo", rank=rank, world_size=world)

    def allreduce_max(x):
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    timer = bench.Timer(world, lambda: None, dist.barrier, allreduce_max)
    # rank 1 is slower: the reported time must be the slowest rank's, on every rank
    elapsed = timer.run(lambda: time.sleep(0.02 * (1 + rank)), 3)
    unc, rx = synth.make_frames(7, bench.G, 8, 64, soft=True, seed=bench.shard_seed(rank))
    q.put((rank, elapsed, unc.tobytes()))
    dist.destroy_process_group()


def test_two_rank_timer_and_shards():
    import bench

    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, t0, u0), (r1, t1, u1) = res
    assert t0 == t1  # max over ranks, identical everywhere
    assert t0 >= 3 * 0.04  # at least the slow rank's own time
    assert u0 != u1  # disjoint shards
    assert bench.shard_seed(0) != bench.shard_seed(1)


def test_shard_seed_reproducible():
    import bench
    from convolutionalencdec_amd import synth

    a = synth.make_frames(7, bench.G, 4, 32, soft=False, seed=bench.shard_seed(3))
    b = synth.make_frames(7, bench.G, 4, 32, soft=False, seed=bench.shard_seed(3))
    assert all(np.array_equal(x, y) for x, y in zip(a, b))
