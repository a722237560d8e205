"""Measurement only: vtb_decode_host_multi (plan per call) against a persistent plan's
vtb_decode_host on the same host batch."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from convolutionalencdec_amd import ConvCode, ViterbiDecoder, decode_multi, synth  # noqa: E402

for F in (4096, 65536):
    code = ConvCode(7, (0o113, 0o171))
    unc, rx = synth.make_frames(7, (0o113, 0o171), F, 1024, soft=True, snr_db=-5.0, seed=5)
    x = np.ascontiguousarray(rx.reshape(F, -1))
    dec = ViterbiDecoder(code, frame_bits=1024, soft=True)
    for name, fn in (("plan", lambda: dec.decode_host(x)), ("multi", lambda: decode_multi(x, code, 1024, soft=True))):
        fn()
        t = time.perf_counter()
        for _ in range(10):
            out = fn()
        dt = (time.perf_counter() - t) / 10
        print(f"F={F} {name}: {dt * 1e6:.0f} us per call, {F * 1024 / dt / 1e9:.2f} Gbit/s")
