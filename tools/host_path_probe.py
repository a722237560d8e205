"""Measurement only: end-to-end (PCIe-inclusive) decode rates for host-resident frames.
Pageable numpy buffers through vtb_decode_host vs pinned torch buffers with the copies and
the kernel on one stream, and with chunked copy/compute overlap on two streams."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from convolutionalencdec_amd import ConvCode, ViterbiDecoder, synth  # noqa: E402

F, L = int(sys.argv[1]) if len(sys.argv) > 1 else 4096, 1024
unc, rx = synth.make_frames(7, (0o113, 0o171), F, L, soft=True, snr_db=-5.0, seed=5)
x_np = np.ascontiguousarray(rx.reshape(F, -1))
dec = ViterbiDecoder(ConvCode(7, (0o113, 0o171)), frame_bits=L, soft=True)
ib, ob = x_np.shape[1], L // 8


def rate(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / reps
    return F * L / dt / 1e9, dt * 1e6


print("pageable vtb_decode_host: %.2f Gbit/s (%.0f us)" % rate(lambda: dec.decode_host(x_np)))
h_in = torch.from_numpy(x_np).pin_memory()
h_out = torch.empty((F, ob), dtype=torch.uint8).pin_memory()
d_in = torch.empty((F, ib), dtype=torch.uint8, device="cuda")
d_out = torch.empty((F, ob), dtype=torch.uint8, device="cuda")


def pinned_serial():
    d_in.copy_(h_in, non_blocking=True)
    dec.decode_device(d_in, out=d_out)
    h_out.copy_(d_out, non_blocking=True)
    torch.cuda.current_stream().synchronize()


print("pinned serial: %.2f Gbit/s (%.0f us)" % rate(pinned_serial))


def h2d_only():
    d_in.copy_(h_in, non_blocking=True)
    torch.cuda.current_stream().synchronize()


print("pinned H2D only: %.2f Gbit/s-equiv (%.0f us), %.1f GB/s" % (*rate(h2d_only), F * ib / rate(h2d_only)[1] / 1e3))
for nch in (2, 4, 8):
    cs, ks, ds = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
    per = (F + nch - 1) // nch
    decs = dec

    def pipelined():
        evs = []
        for i in range(nch):
            lo, hi = i * per, min(F, (i + 1) * per)
            with torch.cuda.stream(cs):
                d_in[lo:hi].copy_(h_in[lo:hi], non_blocking=True)
                e = torch.cuda.Event()
                e.record(cs)
            ks.wait_event(e)
            decs.decode_device(d_in[lo:hi], out=d_out[lo:hi], stream=ks.cuda_stream)
            e2 = torch.cuda.Event()
            e2.record(ks)
            with torch.cuda.stream(ds):
                ds.wait_event(e2)
                h_out[lo:hi].copy_(d_out[lo:hi], non_blocking=True)
        ds.synchronize()

    print("pinned pipelined %d chunks: %.2f Gbit/s (%.0f us)" % (nch, *rate(pipelined)))
ref = dec.decode_host(x_np)
assert (h_out.numpy() == ref).all()
print("outputs identical")
