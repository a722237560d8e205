"""Measurement only: phase timestamps of the generic single-frame kernel (gen_seg_kernel,
Launch::tstamp) on one frame decoded through vtb_decode_frame_sync.

    python tools/tstamp_seg.py [--K 3,4,5,6,8] [--frame-bits 2048] [--reps 50] [--soft]

Per K: median microseconds of each phase (staging, steps, boundary checks (with the wait for the
other waves), the verified traceback with its bytes, output) and the core clock (GHz) over the
kernel.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

# (phase name, start entry, end entry) of the kernel's timestamps (gen_seg_kernel ts(k))
PHASES = (("stage", 0, 1), ("steps", 1, 2), ("check", 2, 3), ("traceback", 3, 5), ("output", 5, 6))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", default="3,4,5,6,8")
    ap.add_argument("--frame-bits", type=int, default=2048)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--soft", action="store_true")
    a = ap.parse_args()
    import torch

    from convolutionalencdec_amd import ConvCode, ViterbiDecoder, native
    from helpers import LENGTH_CODES, encode_bits, hard_to_soft

    codes = {K: g for name, (K, g) in LENGTH_CODES.items() if name != "k3"}  # (k3: the non-symmetric code)
    lib = native.lib()
    lib.vtb_debug_set_tstamp.argtypes = [ctypes.c_void_p]
    buf = torch.zeros(8, dtype=torch.int64, device="cuda")
    for K in (int(k) for k in a.K.split(",")):
        g = codes[K]
        rng = np.random.default_rng(314)
        unc = rng.integers(0, 2, a.frame_bits, dtype=np.uint8)
        coded = np.ascontiguousarray(encode_bits(K, g, unc[None, :])[0])
        x = hard_to_soft(coded[None, :])[0] if a.soft else coded
        d = ViterbiDecoder(ConvCode(K, g), frame_bits=a.frame_bits, soft=a.soft)
        for _ in range(5):
            d.decode_frame(x)
        rows = []
        for _ in range(a.reps):
            buf.zero_()
            torch.cuda.synchronize()
            lib.vtb_debug_set_tstamp(ctypes.c_void_p(buf.data_ptr()))
            d.decode_frame(x)
            lib.vtb_debug_set_tstamp(None)
            torch.cuda.synchronize()
            b = buf.cpu().numpy().astype(np.int64)
            if b[0] != 0 and b[6] != 0:
                rows.append(b)
        if not rows:
            print(json.dumps({"K": K, "note": "no gen_seg launch recorded", "kernel": native.last_kernel()}))
            continue
        b = np.array(rows)
        ph = {n: float(np.median(b[:, j] - b[:, i])) * 0.01 for n, i, j in PHASES}
        ghz = float(np.median(b[:, 7] / np.maximum(b[:, 6] - b[:, 0], 1))) / 10.0
        print(json.dumps({"K": K, "L": a.frame_bits, "soft": a.soft, "n": len(rows),
                          "total_us": round(float(np.median(b[:, 6] - b[:, 0])) * 0.01, 2),
                          "phases_us": {k: round(v, 2) for k, v in ph.items()}, "clock_ghz": round(ghz, 2)}),
              flush=True)
        d.close()


if __name__ == "__main__":
    main()
