"""Measurement only: general rate-k/n decoder time against the frame count (is a code
latency-bound -- time flat in frames -- or throughput-bound?).  $FRAMES: comma-separated frame
counts; with $VTB_DEBUG=1 / 2 the kernel skips its traceback / its ACS (the split of the time)."""
import json
import os
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from helpers import GENK_CODES  # noqa: E402

from convolutionalencdec_amd import GenKDecoder  # noqa: E402

for k, K, g in GENK_CODES:
    L = 1024 if k == 1 else 1032
    d = GenKDecoder(k, K, g, L)
    for F in [int(v) for v in os.environ.get("FRAMES", "1024,4096,16384,65536").split(",")]:
        x = torch.randint(0, 1 << len(g), (F, d.in_bytes), dtype=torch.uint8, device="cuda")
        out = torch.empty((F, d.out_bytes), dtype=torch.uint8, device="cuda")
        for _ in range(2):
            d.decode_device(x, out)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            d.decode_device(x, out)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 5
        print(json.dumps({"k": k, "K": K, "n": len(g), "frames": F, "kernel_ms": round(ms, 4),
                          "mbit_s": round(F * L / ms / 1e3, 1)}), flush=True)
