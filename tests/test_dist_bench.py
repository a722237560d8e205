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


class _Args:
    def __init__(self, **kw):
        self.gpus, self.source = 1, "rank"
        self.__dict__.update(kw)


@pytest.mark.parametrize("gpus,env,source,mode", [
    (1, {}, "rank", "run"),
    (8, {}, "rank", "spawn"),  # `bench.py --gpus 8` alone starts 8 ranks, never times one GPU as 8
    (8, {"WORLD_SIZE": "8"}, "rank", "run"),  # the driver's torchrun form
    (8, {"WORLD_SIZE": "4"}, "rank", "error"),  # a mismatch is refused, not reported as n_gpus 4 or 8
    (2, {"WORLD_SIZE": "1"}, "rank", "error"),
    (8, {}, "gpu0", "run"),  # one process drives every GPU over xGMI
    (8, {"WORLD_SIZE": "8"}, "gpu0", "error"),
    (0, {}, "rank", "error"),
])
def test_launch_decision(gpus, env, source, mode):
    import bench

    plan = bench.launch_plan(_Args(gpus=gpus, source=source), env, ["--gpus", str(gpus)], port=12345)
    assert plan["mode"] == mode, plan
    if mode == "spawn":
        cmd = plan["cmd"]
        assert cmd[1:3] == ["-m", "torch.distributed.run"]
        assert f"--nproc-per-node={gpus}" in cmd and "127.0.0.1" in cmd
        assert cmd[-2:] == ["--gpus", str(gpus)]


def test_spawned_ranks_see_their_world(tmp_path):
    """The spawn path end to end on CPU: the torchrun command bench.py would start, with
    --dry-run added, runs two ranks that each decide 'run' with world 2 (no GPU touched)."""
    import json
    import subprocess

    import bench

    argv = ["--gpus", "2", "--dry-run"]
    plan = bench.launch_plan(bench.parse(argv), {}, argv, port=_free_port())
    assert plan["mode"] == "spawn"
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run(plan["cmd"], capture_output=True, text=True, timeout=180, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 2 and all(ln["mode"] == "run" and ln["world"] == 2 for ln in lines), r.stdout


def test_bench_exits_nonzero_on_world_mismatch():
    import subprocess

    env = dict(os.environ, WORLD_SIZE="4", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "8"], capture_output=True,
                       text=True, timeout=120, env=env)
    assert r.returncode == 2 and "WORLD_SIZE=4" in r.stderr


@pytest.mark.parametrize("F,G", [(1 << 20, 8), (4096, 3), (7, 8), (1000003, 7)])
def test_strong_split_matches_the_c_abi(F, G):
    """bench.py's --global-frames shards are vtb_shard_range's (a host-only C ABI call)."""
    import bench
    from convolutionalencdec_amd import shard_range

    bounds = [bench.shard_bounds(F, G, i) for i in range(G)]
    assert bounds[0][0] == 0 and bounds[-1][1] == F
    assert all(bounds[i][1] == bounds[i + 1][0] for i in range(G - 1))
    assert max(h - lo for lo, h in bounds) - min(h - lo for lo, h in bounds) <= 1
    try:
        native_bounds = [shard_range(F, G, i) for i in range(G)]
    except OSError:  # pragma: no cover - the library needs the ROCm runtime to load
        pytest.skip("libviterbi_amd.so not loadable here")
    assert bounds == native_bounds
    args = bench.parse(["--global-frames", str(F), "--gpus", str(G)])
    assert sum(bench.frames_for_rank(args, G, r) for r in range(G)) == F
