"""Measurement only: N synchronous single-frame decodes (vtb_decode_frame_sync) of one
noiseless frame, for rocprofv3 --kernel-trace --stats; VTB_DEBUG selects skipped phases.

    python tools/probes/frame_phases.py K L N"""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from convolutionalencdec_amd import ConvCode, ViterbiDecoder, frames  # noqa: E402

CODES = {7: (0o113, 0o171), 9: (0o561, 0o753)}
K, L, N = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
code = ConvCode(K, CODES[K])
unc, rx = frames.make_frames(code, 1, L, soft=False, p=0.0, seed=1)
x = rx.reshape(1, -1)[0].cpu().numpy()
d = ViterbiDecoder(code, frame_bits=L)
ok = (d.decode_frame(x) == unc.cpu().numpy()[0]).all()
t0 = time.perf_counter()
for _ in range(N):
    d.decode_frame(x)
dt = time.perf_counter() - t0
print(f"K={K} L={L}: {dt / N * 1e6:.1f} us per call (python loop), first frame correct={ok}")
