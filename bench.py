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

Launch modes (launch_plan; `--dry-run` prints the decision without touching a GPU):
  * under torchrun (WORLD_SIZE set): one rank per GPU; WORLD_SIZE must equal --gpus.
  * `--gpus N` (N > 1) without WORLD_SIZE: this process starts torchrun with N ranks as a
    child (before any HIP call) and exits with its status, so `bench.py --gpus 8` alone
    measures 8 GPUs, never silently one.
  * `--global-frames G`: strong split of one G-frame batch, rank r decodes frames
    [floor(G r / N), floor(G (r+1) / N)) (vtb_shard_range), e.g. config C5 = 2^20 frames.
  * `--source gpu0`: one process; the whole batch is resident on GPU 0 and each step is one
    vtb_decode_peer_multi call that scatters the shards over xGMI, decodes them on every GPU
    and gathers the bytes back (SURVEY.md 8 e, the GPU0-sourced C5 variant).
"""
import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "decoded info Mbit/s, K=7 r=1/2 soft-dec, batch 4096 frames @1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
K, G = 7, (0o113, 0o171)
# every k = 1 rate-1/2 constraint length (K = 3, 4, 6, 8: the generic kernel; params/k<K>)
CODES = {3: (3, (0o7, 0o5)), 4: (4, (0o15, 0o17)), 5: (5, (0o23, 0o35)), 6: (6, (0o53, 0o75)), 7: (7, G),
         8: (8, (0o247, 0o371)), 9: (9, (0o561, 0o753))}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--frames", type=int, default=4096, help="frames per GPU")
    ap.add_argument("--frame-bits", type=int, default=1024)
    ap.add_argument("--hard", action="store_true", help="hard-decision input instead of 8-bit soft")
    ap.add_argument("--K", type=int, default=7, choices=tuple(range(3, 10)))
    ap.add_argument("--snr-db", type=float, default=-5.0)
    ap.add_argument("--cpu-seconds", type=float, default=8.0, help="CPU baseline wall time (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU baseline threads (0 = the effective CPUs: min(affinity mask, cgroup quota))")
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
    ap.add_argument("--gen", choices=("auto", "host", "device"), default="auto",
                    help="synthetic frames from numpy on the host or from the device generator (csrc/vtb_gen.hip: "
                         "no PCIe); auto = host up to 16,384 frames per GPU, device beyond")
    ap.add_argument("--global-frames", type=int, default=0,
                    help="strong split: one batch of this many frames over all GPUs (rank r gets frames "
                         "[G r / N, G (r+1) / N)); 0 = --frames per GPU (weak scaling)")
    ap.add_argument("--source", choices=("rank", "gpu0"), default="rank",
                    help="rank: every rank generates and decodes its own shard; gpu0: one process, the batch "
                         "resident on GPU 0, shards scattered over xGMI by vtb_decode_peer_multi each step")
    ap.add_argument("--peer-devices", default="",
                    help="--source gpu0: comma-separated device list (default 0..N-1; repeats allowed, e.g. "
                         "0,0 to rehearse the staged path on one GPU)")
    ap.add_argument("--peer-stage-all", action="store_true",
                    help="--source gpu0: stage every shard through its own buffers and peer copies "
                         "(VTB_PEER_STAGE_ALL), the source GPU's too")
    ap.add_argument("--dry-run", action="store_true",
                    help="print the launch decision (and the torchrun command it would start) as JSON and exit")
    return ap.parse_args(argv)


def dist_env(environ=None):
    environ = os.environ if environ is None else environ
    world = int(environ.get("WORLD_SIZE", "1"))
    rank = int(environ.get("RANK", "0"))
    local = int(environ.get("LOCAL_RANK", "0"))
    return world, rank, local


def free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def debug_bits_dropped(environ):
    """True (with a message) when $VTB_DEBUG asks for phase-timing bits the loaded library does
    not honour: the shipped build masks the output-corrupting bits 0-4 (vtb_internal.h
    kDbgUnsafe), so a phase-timing script run without VTB_LIB_PATH pointing at a -DVTB_MEASURE
    build (tools/build_variants.sh) would time the full kernel and report it as a phase."""
    want = environ.get("VTB_DEBUG", "")
    if not want:
        return False
    from convolutionalencdec_amd import native

    try:
        req = int(want)
    except ValueError:
        req = 0
    got = native.effective_debug_flags()
    if got == req:
        return False
    print(f"bench.py: VTB_DEBUG={req} but the loaded library ({native.LIB_PATH}) honours {got}: the "
          "phase-timing bits 0-4 need a -DVTB_MEASURE build (tools/build_variants.sh, VTB_LIB_PATH)",
          file=sys.stderr, flush=True)
    return True


def launch_plan(args, environ, argv, port=None):
    """What this invocation does, decided before any HIP call:
    {"mode": "run" | "spawn" | "error", "world": N, "reason": ..., "cmd": [...] (spawn)}."""
    ws = environ.get("WORLD_SIZE")
    if args.gpus < 1:
        return {"mode": "error", "world": 0, "reason": f"--gpus {args.gpus} < 1"}
    if args.source == "gpu0":
        if ws is not None and int(ws) != 1:
            return {"mode": "error", "world": int(ws),
                    "reason": "--source gpu0 is one process driving every GPU; do not launch it under torchrun"}
        return {"mode": "run", "world": 1, "reason": f"one process, GPU 0 scatters to {args.gpus} GPU(s) over xGMI"}
    if ws is not None:
        if int(ws) != args.gpus:
            return {"mode": "error", "world": int(ws),
                    "reason": f"WORLD_SIZE={ws} but --gpus {args.gpus}: refusing to report a different GPU count"}
        return {"mode": "run", "world": int(ws), "reason": "rank of an external torchrun launch"}
    if args.gpus == 1:
        return {"mode": "run", "world": 1, "reason": "one GPU, one process"}
    port = free_port() if port is None else port
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)
    return {"mode": "spawn", "world": args.gpus, "reason": f"--gpus {args.gpus} without WORLD_SIZE: starting "
                                                            f"{args.gpus} ranks under torchrun", "cmd": cmd}


def shard_bounds(frames, shards, index):
    """[lo, hi) of shard `index`: floor(F i / G) .. floor(F (i+1) / G), the split of
    vtb_shard_range (include/viterbi_amd.h)."""
    def bound(i):
        return (frames // shards) * i + (frames % shards) * i // shards
    return bound(index), bound(index + 1)


def frames_for_rank(args, world, rank):
    if args.global_frames > 0:
        lo, hi = shard_bounds(args.global_frames, world, rank)
        return hi - lo
    return args.frames


def use_device_gen(args, frames):
    return args.gen == "device" or (args.gen == "auto" and frames > 16384)


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


def effective_cpus():
    """(CPUs this process may run on, CPUs' worth of time it may use): min(affinity mask,
    cgroup quota rounded up), and the affinity count itself."""
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        avail = os.cpu_count() or 1
    quota = cgroup_cpus()
    eff = avail if quota is None else max(1, min(avail, int(-(-quota // 1))))
    return eff, avail


def cpu_flags():
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("flags"):
                    return set(line.split(":", 1)[1].split())
    except OSError:  # pragma: no cover
        pass
    return set()


AVX512_V4 = {"avx512f", "avx512bw", "avx512dq", "avx512vl", "avx512cd"}


def ref_builds():
    """The reference decoder builds this host can run: x86-64-v3 (AVX2) always, x86-64-v4
    (AVX-512) when the CPU has its flags (oracle/Makefile)."""
    d = os.path.join(REPO, "oracle", "_ref")
    out = [("x86-64-v3 (AVX2)", os.path.join(d, "libref_k7.so"))]
    if AVX512_V4 <= cpu_flags():
        out.append(("x86-64-v4 (AVX-512)", os.path.join(d, "libref_k7_v4.so")))
    return [(isa, p) for isa, p in out if os.path.exists(p)]


def cpu_baseline(seconds, threads, frame_bits):
    """Reference decoder (oracle/_ref/libref_k7*.so, compiled from the reference sources) on
    this host: the speedDecode protocol (speedDecode.c:37-116) with the workload's frame
    length, one independent decoder state per thread.  The reference's own recipe is -Ofast
    -march=native (speedDecode/Makefile:4); the sources do not travel to the GPU box, so both
    prebuilt ISA levels the host supports are probed for one second on one core and the faster
    one runs the timed sample.  Threads default to the effective CPUs (min of the affinity
    mask and the cgroup quota).  Falls back to the oracle port."""
    pkt_bytes = frame_bits // 8
    eff, avail = effective_cpus()
    threads = eff if threads <= 0 else max(1, min(threads, avail))
    builds = ref_builds()
    if builds:
        # The reference's VITERBI_INIT prints to stdout; keep stdout for the one JSON line.
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            probes = []
            for isa, path in builds:
                lib = ctypes.CDLL(path)
                lib.ref_speed.restype = ctypes.c_double
                lib.ref_speed.argtypes = [ctypes.c_double, ctypes.c_int, ctypes.c_int]
                probes.append((lib.ref_speed(1.0, 1, pkt_bytes), isa, lib))
            one, isa, lib = max(probes, key=lambda p: p[0])
            mbps = lib.ref_speed(seconds, threads, pkt_bytes)
            # also one core at speedDecode's own 2048-bit packets (speedDecode.c:38-47)
            one_2048 = lib.ref_speed(min(2.0, seconds), 1, 256)
        finally:
            os.dup2(saved, 1)
            os.close(saved)
        return {"value": round(mbps, 2), "unit": "Mbit/s", "cores": threads, "kind": "reference", "isa": isa,
                "isa_probe_single_core": {p[1]: round(p[0], 2) for p in probes},
                "single_core_value": round(one, 2), "single_core_value_2048bit": round(one_2048, 2),
                "cpu_model": cpu_model(), "host_cpus_available": avail, "cgroup_cpu_quota": cgroup_cpus(),
                "effective_cpus": eff,
                "sample": f"reference viterbiDecoderHardButterflyk1 (hard; the reference has no soft decoder), K=7, "
                          f"{frame_bits}-bit frames, speedDecode protocol (16 packets, srand(314)), {threads} threads x "
                          f"{seconds:g} s, one decoder state per thread, {isa} build"}
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
            "effective_cpus": eff, "host_cpus_available": avail,
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


def load_kernel_time(workload_key):
    """rocprofv3 --kernel-trace --stats average duration of the decode kernel on this library
    (profiles/kernel_time.json, tools/kernel_time_summary.py): {"avg_ns", "kernel", "calls"}."""
    ent = _stamped("kernel_time.json", workload_key)
    return ent if ent is not None and isinstance(ent.get("avg_ns"), (int, float)) else None


# VALU issue peaks.  The SIMD-32's full rate, a wave64 instruction every 2 cycles
# (MI355X_MICROARCH.md:54), at the 2.4 GHz peak engine clock over 256 CUs x 4 SIMDs: the
# absolute peak `roofline.secondary` reports against.  The 4-cycle rate is what the integer ops
# this path depends on (v_pk_min_u16, DPP adds) issue at; only plain 32-bit ops reach the 2-cycle
# rate, with two or more waves per SIMD (profiles/r01/isa_bench*.txt).  The mix of each kernel's
# ACS loop prices between the two (`issue_priced`, tools/isa_mix.py, profiles/isa_mix.json).
VALU_PEAK_2CYC_G = 256 * 4 * 2.4 / 2
VALU_PEAK_4CYC_G = 256 * 4 * 2.4 / 4

# roofline.secondary.note per kernel instance (vtb_debug_last_kernel)
KERNEL_NOTES = {
    "k7_lds": "K=7 pair kernel (vtb_k7_lds.hip): packed u16 ACS, 2 frames per wave64, survivors in LDS, one wave "
              "per frame pair",
    "k7_lds_loop": "K=7 pair kernel, persistent over frame pairs: packed u16 ACS, 2 frames per wave64, survivors in "
                   "LDS",
    "k7_lds_split": "K=7 split frames: one frame per wave64 as two halves in the u16 halves, survivors in LDS",
    "k7_split_loop": "K=7 persistent split kernel: one frame per wave64 as two halves, survivors in LDS, in-wave "
                     "fix-up, unconverged frames to the list kernel",
    "k7_global": "K=7 pair kernel with survivor words in a global workspace (newest steps in LDS for hard input)",
    "k7_global_loop": "K=7 pair kernel, persistent, survivor words in a global workspace",
    "k9": "K=9 frame kernel (vtb_k9.hip): 4 metric registers per lane, 2 frames per wave64, survivor words in a "
          "global workspace",
    "k9_loop": "K=9 frame kernel, persistent over frame pairs, survivor words in a global workspace",
    "k9s": "K=9 one frame per wave64 (vtb_k9.hip k9s): 2 metric registers per lane, the frame's 256 locations in "
           "the u16 halves, survivor words in a global workspace",
    "lds_path": "generic K=3..9 kernel (vtb_lds_path.hip): int32 metrics in a register-resident trellis (DPP / permlane partners)",
}


def load_isa_mix(kernel, soft):
    """The issue-priced VALU bound of `kernel`'s ACS loop on this library (profiles/isa_mix.json,
    tools/isa_mix.py), or None."""
    return _stamped("isa_mix.json", f"{kernel}/{'soft' if soft else 'hard'}")


def secondary_block(avg_ms, state_steps, kernel, valu=None, mix=None):
    """roofline.secondary: the bound that holds, integer VALU issue.  achieved = the PMC-counted
    wave64 VALU instructions per launch / avg_ms, against the 2-cycle peak (`frac`), the 4-cycle
    rate (`frac_4cycle`) and the kernel's issue-priced ACS mix (`issue_priced`)."""
    sec = {"bound": "valu", "kernel": kernel,
           "note": KERNEL_NOTES.get(kernel, "see DESIGN.md 5") + "; DESIGN.md 5",
           "state_steps_per_s": round(state_steps / (avg_ms * 1e-3))}
    ach = None
    if valu:
        ach = valu["valu_wave_insts_per_launch"] / (avg_ms * 1e-3) / 1e9
        sec.update({"achieved": round(ach, 2), "unit": "G wave64-VALU-instr/s",
                    "peak": VALU_PEAK_2CYC_G, "frac": round(ach / VALU_PEAK_2CYC_G, 4),
                    "peak_note": "2-cycle wave64 issue (MI355X_MICROARCH.md:54), 1,024 SIMDs at 2.4 GHz",
                    "peak_4cycle": VALU_PEAK_4CYC_G, "frac_4cycle": round(ach / VALU_PEAK_4CYC_G, 4),
                    "valu_wave_insts_per_launch": valu["valu_wave_insts_per_launch"]})
    if mix:
        ip = {"peak": mix["priced_peak_G"], "valu_per_wave_step": mix["valu_per_wave_step"],
              "priced_cycles_per_wave_step": mix["priced_cycles_per_wave_step"],
              "note": "the ACS loop's own instruction mix priced at the measured issue costs (2.8 / 4.6 / 9.4 "
                      "cycles: plain / packed, DPP, VOP3 / permlane swap; tools/isa_mix.py); the launch also "
                      "holds the traceback"}
        if ach is not None:
            ip["frac"] = round(ach / mix["priced_peak_G"], 4)
        sec["issue_priced"] = ip
    return sec


def roofline_block(alg_bytes, avg_ms, n_avg, kern_ms, launch_ms, issue_us, state_steps, kernel, traffic=None,
                   kernel_time=None, valu=None, mix=None):
    """The bench line's `roofline` object.  HBM roofline of the decode kernel: algorithmic bytes
    per launch / the average launch time avg_ms (back-to-back launches) against
    8 TB/s, `traffic` = PMC-measured HBM bytes per launch.  `secondary`: the bound that holds,
    integer VALU issue, against the 2-cycle peak and the kernel's issue-priced mix."""
    achieved = alg_bytes / (avg_ms * 1e-3) / 1e9
    sec = secondary_block(avg_ms, state_steps, kernel, valu, mix)
    issue_bound = issue_us is not None and issue_us * 1e-3 >= 0.8 * avg_ms
    return {
        "bound": "hbm",
        "achieved": round(achieved, 3),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 6),
        "traffic": traffic,
        "kernel_avg_ms": round(avg_ms, 5),
        "kernel_avg_note": f"HIP events around {n_avg} back-to-back launches on the launch stream, opened behind a "
                           "running launch (no first-launch latency); achieved/frac use it",
        "kernel_avg_issue_bound": issue_bound,
        "rocprof_avg_ms": round(kernel_time["avg_ns"] * 1e-6, 5) if kernel_time else None,
        "timed_span_ms": round(kern_ms, 5),
        "timed_span_note": "event span of the timed region / steps; opens on an idle stream, so it includes the "
                           "first launch's dispatch latency",
        "per_launch_pass_ms": {"min": round(min(launch_ms), 5), "median": round(float(np.median(launch_ms)), 5),
                               "max": round(max(launch_ms), 5), "first": round(launch_ms[0], 5),
                               "note": "untimed pass after the timed region, an event after every launch"},
        "host_issue_us_per_launch": round(issue_us, 2) if issue_us is not None else None,
        "algorithmic_bytes_per_launch": alg_bytes,
        # the path is integer-VALU bound (add-compare-select), not HBM bound: SURVEY.md 8(d)
        "secondary": sec,
    }


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


def peer_bench(args):
    """--source gpu0: the batch is resident on GPU 0 (produced there by the device generator,
    as by a demodulator) and each step is one vtb_decode_peer_multi call: shard i of the
    devices list is copied to its GPU over xGMI, decoded there on that GPU's own stream and
    plan, and its L/8 bytes per frame copied back; GPU 0's own shard decodes in place.  The
    call is asynchronous on GPU 0's current stream, whose completion covers every shard.
    value = all frames' bits / step time (strong scaling over the devices list)."""
    import torch

    from convolutionalencdec_amd import ConvCode, decode_peer
    from convolutionalencdec_amd import frames as devframes

    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a ROCm GPU")
    devs = [int(d) for d in args.peer_devices.split(",")] if args.peer_devices else list(range(args.gpus))
    if not devs or any(d < 0 or d >= torch.cuda.device_count() for d in devs):
        raise SystemExit(f"--peer-devices {devs}: {torch.cuda.device_count()} GPU(s) visible")
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    code = ConvCode(*CODES[args.K])
    soft = not args.hard
    L = args.frame_bits
    G_frames = args.global_frames if args.global_frames > 0 else args.frames * len(devs)
    d_unc, d_rx = devframes.make_frames(code, G_frames, L, soft=soft, snr_db=args.snr_db, p=0.0559,
                                        seed=shard_seed(0), device=0)
    x = d_rx.reshape(G_frames, -1)
    out = torch.empty((G_frames, (L + 7) // 8), dtype=torch.uint8, device=dev)

    def step():
        decode_peer(x, devs, code=code, frame_bits=L, soft=soft, out=out, stage_all=args.peer_stage_all)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    ref = out.clone()
    timer = Timer(1, lambda: torch.cuda.synchronize(dev), lambda: None, lambda t: t)
    stream = torch.cuda.current_stream(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    elapsed = timer.run(step, args.steps, on_start=lambda: ev0.record(stream), on_end=lambda: ev1.record(stream))
    call_ms = ev0.elapsed_time(ev1) / args.steps
    same = bool(torch.equal(out, ref))
    ber = float(np.unpackbits((out ^ d_unc).cpu().numpy()).mean())
    T = L + code.S
    in_b = (2 if soft else 1) * T
    ob = (L + 7) // 8
    remote = sum(hi - lo for i, d in enumerate(devs) for lo, hi in [shard_bounds(G_frames, len(devs), i)]
                 if d != 0 or args.peer_stage_all)
    value = G_frames * L / (elapsed / args.steps) / 1e6
    alg = G_frames * (in_b + ob)
    line = {"metric": METRIC, "value": round(value, 2), "unit": "Mbit/s", "n_gpus": len(set(devs)),
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 5),
            "higher_is_better": True, "scaling": "strong" if args.global_frames > 0 else "weak",
            "vs_baseline": None, "dtype": "u16", "data": "synthetic (device generator on GPU 0)",
            "config": {"workload": f"K={args.K} r=1/2 {'8-bit soft' if soft else 'hard'}-decision Viterbi, "
                                   f"{G_frames} frames x {L} info bits resident on GPU 0, shards over "
                                   f"{len(devs)} device slot(s) {devs} via xGMI (vtb_decode_peer_multi)",
                       "global_batch_frames": G_frames, "frame_bits": L, "devices": devs,
                       "stage_all": bool(args.peer_stage_all),
                       "parallelism": "GPU0-sourced contiguous shards, peer copies, no collective",
                       "xgmi_bytes_per_step": remote * (in_b + ob), "outputs_stable": same, "decoded_ber": ber},
            "roofline": {"bound": "hbm", "achieved": round(alg / (call_ms * 1e-3) / 1e9, 3), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(alg / (call_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 6),
                         "traffic": None, "kernel_ms": round(call_ms, 5), "algorithmic_bytes_per_launch": alg,
                         "note": "kernel_ms spans one whole peer call on GPU 0's stream (copies + every shard's "
                                 "decode), not one kernel"},
            "cpu_baseline": None}
    print(json.dumps(line), flush=True)
    return 0


def main():
    argv = sys.argv[1:]
    args = parse(argv)
    plan = launch_plan(args, os.environ, argv)
    if args.dry_run:
        print(json.dumps(plan), flush=True)
        return 0
    if plan["mode"] == "error":
        print(f"bench.py: {plan['reason']}", file=sys.stderr, flush=True)
        return 2
    if plan["mode"] == "spawn":
        # a child process (never exec: nothing here has touched the GPU, but the ranks must be
        # torchrun's children so that it can tear them down); our exit status is theirs
        print(f"bench.py: {plan['reason']}", file=sys.stderr, flush=True)
        return subprocess.call(plan["cmd"])
    if debug_bits_dropped(os.environ):
        return 2
    if args.source == "gpu0":
        return peer_bench(args)
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
    F, L = frames_for_rank(args, world, rank), args.frame_bits
    if F < 1:
        raise SystemExit(f"rank {rank}: empty shard ({args.global_frames} frames over {world} GPUs)")
    T = L + code[0] - 1
    device_gen = use_device_gen(args, F)
    if device_gen:
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

    # Average kernel duration for the roofline (untimed, after the timed region): the timed
    # span above opens on an idle stream, so it includes the first launch's dispatch latency.
    # Here ev0 is recorded behind a launch that is still running, so it completes when that
    # kernel ends and the span holds only back-to-back kernels (plus the one gap ev0 opens,
    # spread over at least 50 launches).  rocprofv3's average for the same library, when
    # profiles/kernel_time.json holds one, is reported beside it.
    n_avg = max(args.steps, 50)
    one()
    ev0.record(stream)
    for _ in range(n_avg):
        one()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    avg_ms = ev0.elapsed_time(ev1) / n_avg

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
    if not device_gen:
        rx_host = np.ascontiguousarray(rx.reshape(F, -1))
        dec.decode_host(rx_host)
        reps = 10
        barrier()
        th = time.perf_counter()
        for _ in range(reps):
            dec.decode_host(rx_host)
        host_s = allreduce_max(time.perf_counter() - th)
        host_mbps = round((args.global_frames if args.global_frames > 0 else world * F) * L * reps / host_s / 1e6, 1)

    ms_per_step = elapsed / args.steps * 1e3
    total_frames = args.global_frames if args.global_frames > 0 else F * world
    total_bits = total_frames * L
    value = total_bits / (elapsed / args.steps) / 1e6
    in_b = (2 if soft else 1) * T
    alg_bytes = F * (in_b + (L + 7) // 8)
    workload_key = f"K{code[0]}_{'soft' if soft else 'hard'}_F{F}_L{L}"
    from convolutionalencdec_amd import native

    kernel = native.last_kernel()
    roofline = roofline_block(alg_bytes, avg_ms, n_avg, kern_ms, launch_ms, issue.get("us"),
                              F * (1 << (code[0] - 1)) * T, kernel, traffic=load_traffic(workload_key),
                              kernel_time=load_kernel_time(workload_key), valu=load_valu(workload_key),
                              mix=load_isa_mix(kernel, soft))

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
        "scaling": "strong" if args.global_frames > 0 else "weak",
        "vs_baseline": None,
        "dtype": "u16",
        "data": "synthetic (device generator)" if device_gen else "synthetic",
        "config": {
            "workload": f"K={code[0]} r=1/2 {'8-bit soft' if soft else 'hard'}-decision Viterbi, {F} frames x {L} "
                        f"info bits per GPU, AWGN SNR {args.snr_db:g} dB" if soft else
                        f"K={code[0]} r=1/2 hard-decision Viterbi, {F} frames x {L} info bits per GPU, BSC p=0.0559",
            "frames_per_gpu": F,
            "frame_bits": L,
            "global_batch_frames": total_frames,
            "split": (f"strong: {args.global_frames} frames, contiguous shards (vtb_shard_range)"
                      if args.global_frames > 0 else "weak: --frames per GPU"),
            "parallelism": f"frames sharded over {world} GPU(s), no data-path collective",
            "batches_in_flight": nin,
            "graph": bool(args.graph and nin == 1),
            "host_buffers_mbps": host_mbps,
            "decoded_ber": ber,
        },
        "roofline": roofline,
        "cpu_baseline": cpu,
    }
    print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main() or 0)
