"""Throughput of the general rate-k/n decoder (vtb_genk_decode_device) on device-resident
random hard input (a Viterbi decoder's work does not depend on the data), 4096 frames x
1032 info bits (1024 for k = 1), HIP events on the launch stream.  Measurement only."""
import json
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from helpers import GENK_CODES  # noqa: E402

from convolutionalencdec_amd import GenKDecoder  # noqa: E402

F = 4096
for k, K, g in GENK_CODES:
    L = 1024 if k == 1 else 1032
    d = GenKDecoder(k, K, g, L)
    x = torch.randint(0, 1 << len(g), (F, d.in_bytes), dtype=torch.uint8, device="cuda")
    out = torch.empty((F, d.out_bytes), dtype=torch.uint8, device="cuda")
    for _ in range(3):
        d.decode_device(x, out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    steps = 10
    e0.record()
    for _ in range(steps):
        d.decode_device(x, out)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    nbytes = F * (d.in_bytes + d.out_bytes)
    print(json.dumps({"k": k, "K": K, "n": len(g), "states": 1 << (k * (K - 1)), "frames": F, "info_bits": L,
                      "kernel_ms": round(ms, 4), "mbit_s": round(F * L / ms / 1e3, 1),
                      "hbm_frac": round(nbytes / (ms * 1e-3) / 8e12, 5)}), flush=True)
