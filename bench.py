"""Throughput bench for the MI355X Viterbi decoder (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Workload (BASELINE.json metric "decoded info Mbit/s, K=7 r=1/2 soft-dec, batch 4096
frames"): every rank decodes its own batch of 4096 frames x 1024 information bits of
K=7 {0113, 0171} rate-1/2 code, 8-bit soft input from a BPSK/AWGN channel at SNR -5 dB
(4 sps), inputs resident in HBM before timing starts.  A step = one decode launch over
the rank's batch.  Frames are independent, so ranks share nothing on the data path
(weak scaling, no collective); the only collectives are the timing barrier and the
max-over-ranks reduction of the elapsed time.

Prints ONE JSON line on rank 0 (the driver's contract), with the roofline of the decode
kernel (HIP-event time per launch on the launch stream, algorithmic bytes per launch, HBM
bytes per launch from profiles/pmc_traffic.json) and the CPU baseline (the reference's own
decoder, oracle/_ref, timed on this host's cores at N=1).  dtype "u16": the decoder's path
metrics are packed unsigned 16-bit integers.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "decoded info Mbit/s, K=7 r=1/2 soft-dec, batch 4096 frames @1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
K, G = 7, (0o113, 0o171)
CODES = {5: (5, (0o23, 0o35)), 7: (7, G), 9: (9, (0o561, 0o753))}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--frames", type=int, default=4096, help="frames per GPU")
    ap.add_argument("--frame-bits", type=int, default=1024)
    ap.add_argument("--hard", action="store_true", help="hard-decision input instead of 8-bit soft")
    ap.add_argument("--K", type=int, default=7, choices=(5, 7, 9))
    ap.add_argument("--snr-db", type=float, default=-5.0)
    ap.add_argument("--cpu-seconds", type=float, default=8.0, help="CPU baseline wall time (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU baseline threads (0 = every CPU in this process's affinity mask)")
    ap.add_argument("--inflight", type=int, default=1,
                    help="batches in flight: step i runs on stream i mod inflight (own plan and output), so one "
                         "batch's tail overlaps the next one's start")
    ap.add_argument("--graph", action="store_true",
                    help="launch the K timed steps as one captured HIP graph (K kernel nodes, one batch each) "
                         "instead of K separate launches")
    ap.add_argument("--stream-chunk", type=int, default=0,
                    help="measure the streaming decoder (vtb_stream_*, SURVEY.md 8 f3) instead: every stream "
                         "receives this many segments per step, one long frame per stream")
    ap.add_argument("--dist-backend", choices=("nccl", "gloo"), default="nccl",
                    help="process group for the timing barrier and max-reduction (nccl = RCCL; gloo: rehearsal)")
    ap.add_argument("--gen", choices=("host", "device"), default="host",
                    help="synthetic frames from numpy on the host (default) or from the device generator "
                         "(csrc/vtb_gen.hip: no PCIe, for large batches)")
    return ap.parse_args()


def dist_env():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return world, rank, local


def shard_seed(rank, base=314):
    """Each rank regenerates its own shard from (base seed, rank): disjoint, reproducible."""
    return base + 1000 * rank


class Timer:
    """Barrier + synchronize bracketing; max over ranks (the driver's timing contract)."""

    def __init__(self, world, device_sync, barrier, allreduce_max):
        self.world, self.sync, self.barrier, self.allreduce_max = world, device_sync, barrier, allreduce_max

    def run(self, step, steps, on_start=None, on_end=None):
        self.barrier()
        self.sync()
        t0 = time.perf_counter()
        if on_start:
            on_start()  # e.g. a HIP event on the launch stream (asynchronous, enqueue only)
        for _ in range(steps):
            step()
        if on_end:
            on_end()
        self.sync()
        dt = time.perf_counter() - t0  # this rank's K steps; the closing barrier is not timed
        self.barrier()
        return self.allreduce_max(dt)


def cpu_model():
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:  # pragma: no cover
        pass
    return None


def cgroup_cpus():
    """CPUs' worth of time this process may use (cgroup v2 cpu.max quota / period), or None."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, p = fh.read().split()[:2]
        return None if q == "max" else round(int(q) / int(p), 2)
    except (OSError, ValueError):
        return None


def cpu_baseline(seconds, threads, frame_bits):
    """Reference decoder (oracle/_ref/libref_k7.so, compiled from the reference sources) on
    this host: the speedDecode protocol (speedDecode.c:37-116) with the workload's frame
    length, one independent decoder state per thread.  Falls back to the oracle port."""
    ref = os.path.join(REPO, "oracle", "_ref", "libref_k7.so")
    pkt_bytes = frame_bits // 8
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        avail = os.cpu_count() or 1
    threads = avail if threads <= 0 else max(1, min(threads, avail))
    if os.path.exists(ref):
        lib = ctypes.CDLL(ref)
        lib.ref_speed.restype = ctypes.c_double
        lib.ref_speed.argtypes = [ctypes.c_double, ctypes.c_int, ctypes.c_int]
        # The reference's VITERBI_INIT prints to stdout; keep stdout for the one JSON line.
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            mbps = lib.ref_speed(seconds, threads, pkt_bytes)
            # also one core, at the workload's frame length and at speedDecode's
            # own 2048-bit packets (speedDecode.c:38-47)
            one = lib.ref_speed(min(2.0, seconds), 1, pkt_bytes)
            one_2048 = lib.ref_speed(min(2.0, seconds), 1, 256)
        finally:
            os.dup2(saved, 1)
            os.close(saved)
        return {"value": round(mbps, 2), "unit": "Mbit/s", "cores": threads, "kind": "reference",
                "single_core_value": round(one, 2), "single_core_value_2048bit": round(one_2048, 2),
                "cpu_model": cpu_model(), "host_cpus_available": avail, "cgroup_cpu_quota": cgroup_cpus(),
                "sample": f"reference viterbiDecoderHardButterflyk1 (hard; the reference has no soft decoder), K=7, "
                          f"{frame_bits}-bit frames, speedDecode protocol (16 packets, srand(314)), {threads} threads x "
                          f"{seconds:g} s, one decoder state per thread"}
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from helpers import Oracle  # test infrastructure: the checker, used here only as the timed CPU leg

    from convolutionalencdec_amd import synth

    orc = Oracle()
    frames = 512
    unc, q = synth.make_frames(K, G, frames, frame_bits, soft=True, seed=7)
    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < seconds:
        orc.decode(K, G, q, frame_bits, soft=True, threads=threads)
        n += frames
    dt = time.perf_counter() - t0
    return {"value": round(n * frame_bits / dt / 1e6, 2), "unit": "Mbit/s", "cores": threads, "kind": "port",
            "sample": f"oracle soft decoder (C restatement), {frames} frames x {frame_bits} bits repeated for "
                      f"{seconds:g} s on {threads} threads"}


def lib_sha16():
    """Hash of the shipped decoder library: counter files are only valid for this binary."""
    import hashlib

    with open(os.path.join(REPO, "convolutionalencdec_amd", "lib", "libviterbi_amd.so"), "rb") as fh:
        return hashlib.sha256(fh.read()).hexdigest()[:16]


def _stamped(name, workload_key):
    """Entry `workload_key` of profiles/<name> if it was measured on this exact library
    (tools/traffic_summary.py stamps every entry with lib_sha16), else None: counters of
    another binary are never paired with this run's launch time."""
    try:
        with open(os.path.join(REPO, "profiles", name)) as fh:
            ent = json.load(fh).get(workload_key)
    except (OSError, ValueError):
        return None
    if not isinstance(ent, dict) or ent.get("lib_sha16") != lib_sha16():
        return None
    return ent


def load_traffic(workload_key):
    """HBM bytes per launch measured by the rocprofv3 --pmc passes (profiles/pmc_traffic.json)."""
    ent = _stamped("pmc_traffic.json", workload_key)
    return None if ent is None else ent.get("bytes_per_launch")


def load_valu(workload_key):
    """VALU wave-instructions per launch from the rocprofv3 SQ pass (profiles/pmc_valu.json)."""
    return _stamped("pmc_valu.json", workload_key)


# VALU issue peak: 256 CUs x 4 SIMDs, one wave64 integer VALU instruction per 4 cycles per
# SIMD (v_add_u32 / v_pk_min_u16 / DPP adds: tools/probes/isa_bench.hip, profiles/r01), at the
# 2.4 GHz peak engine clock.
VALU_PEAK_G = 256 * 4 * 2.4 / 4


def stream_bench(args, dev, local, world):
    """Steady-state streaming decode: F streams, one long frame each, C segments per stream
    per step (a step = one vtb_stream_decode call, inputs already in HBM); value = segments
    pushed per second (= decoded bits per second in steady state: the emitted bits trail
    the input by the merge depth)."""
    import torch

    from convolutionalencdec_amd import ConvCode, ViterbiStream
    from convolutionalencdec_amd import frames as devframes

    F, C, soft = args.frames, args.stream_chunk, not args.hard
    steps, warm = args.steps, args.warmup
    L = (steps + warm) * C
    code = ConvCode(*CODES[args.K])
    d_unc, d_rx = devframes.make_frames(code, F, L, soft=soft, snr_db=args.snr_db, p=0.0559,
                                        seed=shard_seed(int(os.environ.get("RANK", "0"))), device=local)
    sb = 2 if soft else 1
    x = d_rx.reshape(F, -1)
    vs = ViterbiStream(code, streams=F, soft=soft, window_steps=max(4 * C, 4096), device=local)
    outs = []

    def push(i, last=False):
        hi = x.shape[1] if last else (i + 1) * C * sb
        o, nb = vs.push(x[:, i * C * sb:hi], last=last)
        outs.append((o, nb))

    for i in range(warm):
        push(i)
    torch.cuda.synchronize(dev)
    stream = torch.cuda.current_stream(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for i in range(warm, warm + steps):
        push(i)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    call_ms = ev0.elapsed_time(ev1) / steps
    push(warm + steps, last=True)  # the tail, untimed
    torch.cuda.synchronize(dev)
    bits = np.concatenate([np.concatenate([np.unpackbits(o[f].cpu().numpy())[:int(nb[f])]
                                           for o, nb in outs]) for f in range(min(F, 8))]).reshape(min(F, 8), -1)
    unc = np.unpackbits(d_unc[:min(F, 8)].cpu().numpy(), axis=1)[:, :L]
    ber = float((bits[:, :L] != unc).mean()) if bits.shape[1] == L else None
    value = F * C * steps / dt / 1e6
    alg = F * (C * sb + C // 8)  # input segments in, decoded bits out (steady state)
    line = {"metric": METRIC, "value": round(value, 2), "unit": "Mbit/s", "n_gpus": 1, "steps": steps, "warmup": warm,
            "ms_per_step": round(dt / steps * 1e3, 5), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "u16", "data": "synthetic (device generator)",
            "config": {"workload": f"streaming K={args.K} r=1/2 {'8-bit soft' if soft else 'hard'}-decision, {F} streams x "
                                   f"{C} segments per call (vtb_stream_decode), one {L}-bit frame per stream",
                       "streams": F, "segments_per_call": C, "decoded_ber_first8": ber},
            "roofline": {"bound": "hbm", "achieved": round(alg / (call_ms * 1e-3) / 1e9, 3), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(alg / (call_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 6), "traffic": None,
                         "kernel_ms": round(call_ms, 5), "algorithmic_bytes_per_launch": alg,
                         "note": "one call = the stream kernel (+ a 2-D carry copy when C is not a multiple of 48)"},
            "cpu_baseline": None}
    print(json.dumps(line), flush=True)


def main():
    args = parse()
    world, rank, local = dist_env()
    import torch

    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a ROCm GPU")
    # VTB_BENCH_ONE_DEVICE=1 (rehearsal of the N > 1 path on a one-GPU box, with
    # --dist-backend gloo): every rank on device 0
    gpu = 0 if os.environ.get("VTB_BENCH_ONE_DEVICE") == "1" else local
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    local = gpu
    if args.stream_chunk > 0:
        if world > 1:
            raise SystemExit("--stream-chunk is a single-GPU measurement")
        return stream_bench(args, dev, local, world)
    if world > 1:
        import torch.distributed as dist

        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
        red_dev = dev if args.dist_backend == "nccl" else torch.device("cpu")

        def barrier():
            dist.barrier()

        def allreduce_max(x):
            t = torch.tensor([x], dtype=torch.float64, device=red_dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            return float(t.item())
    else:
        def barrier():
            pass

        def allreduce_max(x):
            return x

    from convolutionalencdec_amd import ConvCode, ViterbiDecoder, synth

    code = CODES[args.K]
    soft = not args.hard
    F, L = args.frames, args.frame_bits
    T = L + code[0] - 1
    if args.gen == "device":
        from convolutionalencdec_amd import frames as devframes

        d_unc, d_rx = devframes.make_frames(ConvCode(*code), F, L, soft=soft, snr_db=args.snr_db, p=0.0559,
                                            seed=shard_seed(rank), device=local)
        x = d_rx.reshape(F, -1)
        torch.cuda.synchronize(dev)
        unc = d_unc.cpu().numpy()
    else:
        unc, rx = synth.make_frames(code[0], code[1], F, L, soft=soft, snr_db=args.snr_db, p=0.0559,
                                    seed=shard_seed(rank))
        x = torch.from_numpy(rx.reshape(F, -1)).to(dev)
    nin = max(1, args.inflight)
    decs = [ViterbiDecoder(ConvCode(*code), frame_bits=L, soft=soft, device=local) for _ in range(nin)]
    outs = [torch.empty((F, (L + 7) // 8), dtype=torch.uint8, device=dev) for _ in range(nin)]
    stream = torch.cuda.current_stream(dev)
    streams = [stream] + [torch.cuda.Stream(dev) for _ in range(nin - 1)]
    dec, out = decs[0], outs[0]
    # one bound launcher per batch in flight: the C ABI call with its arguments validated once
    # (ViterbiDecoder.bind), so a step costs the host only the launch itself
    launchers = [decs[i].bind(x, outs[i], streams[i].cuda_stream) for i in range(nin)]
    state = {"i": 0}

    def step():
        i = state["i"] % nin
        state["i"] += 1
        launchers[i]()

    # Average launch duration for the roofline: HIP events on the launch stream around the
    # timed region's K back-to-back launches (nothing else is enqueued between them: an event
    # after every launch opens a ~3-6 us gap before the next kernel), and the
    # host's issue time per launch.  Created before the warm-up, and the decoded output is
    # checked after the timed region (the same batch into the same buffer), so the GPU does
    # not sit idle between the warm-up and the timed launches (an idle millisecond makes the
    # next launch ~4 us slower).
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    issue = {}
    timer = Timer(world, lambda: torch.cuda.synchronize(dev), barrier, allreduce_max)

    def check_output():
        for o in outs[1:]:
            assert torch.equal(o, outs[0]) or args.warmup < nin
        d = out.cpu().numpy()
        return d, float(np.unpackbits(d ^ unc).mean())

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if args.graph and nin == 1:
        decoded, ber = check_output()
        # the K steps captured as K kernel nodes of one graph (same batch, same output buffer)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            for _ in range(args.steps):
                dec.decode_device(x, out=out)
        graph.replay()
        torch.cuda.synchronize(dev)
        assert torch.equal(out.cpu(), torch.from_numpy(decoded))
        elapsed = timer.run(graph.replay, 1, on_start=lambda: ev0.record(stream), on_end=lambda: ev1.record(stream))
    else:
        def issued():
            issue["s"] = time.perf_counter()
            ev1.record(stream)

        state["i"] = 0
        # ev0 is enqueued before the timed region opens (the stream is idle after the warm-up
        # synchronisation, so it completes at once; kernel_ms still spans t0 -> first kernel)
        ev0.record(stream)
        t_issue0 = time.perf_counter()
        elapsed = timer.run(step, args.steps, on_end=issued)
        issue["us"] = (issue["s"] - t_issue0) / args.steps * 1e6
    kern_ms = ev0.elapsed_time(ev1) / args.steps

    one = launchers[0]
    if nin > 1:
        # the timed region interleaves streams: time K launches on one stream instead
        ev0.record(stream)
        for _ in range(args.steps):
            one()
        ev1.record(stream)
        torch.cuda.synchronize(dev)
        kern_ms = ev0.elapsed_time(ev1) / args.steps

    # Per-launch spread, measured after the timed region (untimed): the same K launches with an
    # event after each.  Those events add a gap before every next launch, so this pass reads
    # slightly slower per launch than kernel_ms; it shows whether single launches are slow.
    per = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    per[0].record(stream)
    for i in range(args.steps):
        one()
        per[i + 1].record(stream)
    torch.cuda.synchronize(dev)
    launch_ms = [per[i].elapsed_time(per[i + 1]) for i in range(args.steps)]
    _, ber = check_output()

    # PCIe-inclusive rate: the same batch from pageable host memory through
    # vtb_decode_host (H2D copy, decode, D2H copy, synchronise); reported beside, never `value`.
    # Every rank at once (each GPU has its own PCIe link): aggregate over ranks, slowest rank.
    host_mbps = None
    if args.gen == "host":
        rx_host = np.ascontiguousarray(rx.reshape(F, -1))
        dec.decode_host(rx_host)
        reps = 10
        barrier()
        th = time.perf_counter()
        for _ in range(reps):
            dec.decode_host(rx_host)
        host_s = allreduce_max(time.perf_counter() - th)
        host_mbps = round(world * F * L * reps / host_s / 1e6, 1)

    ms_per_step = elapsed / args.steps * 1e3
    total_bits = F * L * world
    value = total_bits / (elapsed / args.steps) / 1e6
    in_b = (2 if soft else 1) * T
    alg_bytes = F * (in_b + (L + 7) // 8)
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
    workload_key = f"K{code[0]}_{'soft' if soft else 'hard'}_F{F}_L{L}"
    traffic = load_traffic(workload_key)
    valu = load_valu(workload_key)
    secondary = {"bound": "valu", "state_steps_per_s": round(F * (1 << (code[0] - 1)) * T / (kern_ms * 1e-3)),
                 "note": "packed u16 ACS, 2 frames per wave64; see DESIGN.md 5"}
    if valu:
        ach = valu["valu_wave_insts_per_launch"] / (kern_ms * 1e-3) / 1e9
        secondary.update({"achieved": round(ach, 2), "peak": VALU_PEAK_G, "unit": "G wave64-VALU-instr/s",
                          "frac": round(ach / VALU_PEAK_G, 4),
                          "valu_wave_insts_per_launch": valu["valu_wave_insts_per_launch"]})

    if rank != 0:
        if world > 1:
            torch.distributed.destroy_process_group()
        return
    cpu = None
    if world == 1 and args.cpu_seconds > 0 and code[0] == 7:
        cpu = cpu_baseline(args.cpu_seconds, args.cpu_threads, L)
    line = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "Mbit/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u16",
        "data": "synthetic" if args.gen == "host" else "synthetic (device generator)",
        "config": {
            "workload": f"K={code[0]} r=1/2 {'8-bit soft' if soft else 'hard'}-decision Viterbi, {F} frames x {L} "
                        f"info bits per GPU, AWGN SNR {args.snr_db:g} dB" if soft else
                        f"K={code[0]} r=1/2 hard-decision Viterbi, {F} frames x {L} info bits per GPU, BSC p=0.0559",
            "frames_per_gpu": F,
            "frame_bits": L,
            "global_batch_frames": F * world,
            "parallelism": f"frames sharded over {world} GPU(s), no data-path collective",
            "batches_in_flight": nin,
            "graph": bool(args.graph and nin == 1),
            "host_buffers_mbps": host_mbps,
            "decoded_ber": ber,
        },
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 3),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 6),
            "traffic": traffic,
            "kernel_ms": round(kern_ms, 5),
            "per_launch_pass_ms": {"min": round(min(launch_ms), 5), "median": round(float(np.median(launch_ms)), 5),
                                   "max": round(max(launch_ms), 5), "first": round(launch_ms[0], 5),
                                   "note": "untimed pass after the timed region, an event after every launch"},
            "host_issue_us_per_launch": round(issue["us"], 2) if "us" in issue else None,
            "algorithmic_bytes_per_launch": alg_bytes,
            # the path is integer-VALU bound (add-compare-select), not HBM bound: SURVEY.md 8(d)
            "secondary": secondary,
        },
        "cpu_baseline": cpu,
    }
    print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
