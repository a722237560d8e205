"""Measurement/debug only: replay one single-frame fuzz case (tests/test_gpu_fuzz.py
test_single_frame_path_vs_oracle) through each decode path and report which path differs
from the oracle, and where.

    python tools/dbg_frame_case.py [--i 1947] [--L 2203] [--K 7] [--hard] [--noise 0.5]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--i", type=int, default=1947)
    ap.add_argument("--L", type=int, default=2203)
    ap.add_argument("--K", type=int, default=7)
    ap.add_argument("--hard", action="store_true")
    ap.add_argument("--noise", type=float, default=0.5)
    ap.add_argument("--frames", type=int, default=3)
    a = ap.parse_args()
    import torch

    from helpers import CODES, Oracle, random_frames  # the checker (test infrastructure)

    from convolutionalencdec_amd import ConvCode, ViterbiDecoder, native

    orc = Oracle()
    soft = not a.hard
    K, L, i = a.K, a.L, a.i
    if soft:
        sigma = {0.0: 0.3, 0.03: 0.56, 0.07: 0.7, 0.5: 4.0}[a.noise]
        unc, x = random_frames(orc, K, L, a.frames, 0.0, 5000 + i, soft=True, sigma=sigma)
    else:
        unc, x = random_frames(orc, K, L, a.frames, a.noise, 5000 + i)
    x = np.ascontiguousarray(x).reshape(a.frames, -1)
    want = orc.decode(K, CODES[K], x, L, soft=soft, threads=8)
    lib = native.lib()
    lib.vtb_debug_seg_stats.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]

    def stats():
        s = (ctypes.c_ulonglong * 3)()
        lib.vtb_debug_seg_stats(s)
        return list(s)

    def diff(got):
        r = []
        for f in range(a.frames):
            gb = np.unpackbits(got[f])[:L]
            wb = np.unpackbits(want[f])[:L]
            bad = np.flatnonzero(gb != wb)
            r.append({"frame": f, "bad_bits": int(bad.size), "first": int(bad[0]) if bad.size else None,
                      "last": int(bad[-1]) if bad.size else None})
        return r

    def run(label, env, mode):
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            d = ViterbiDecoder(ConvCode(K, CODES[K]), frame_bits=L, soft=soft)
            per = []
            if mode == "frame":
                got = []
                for f in range(a.frames):
                    s0 = stats()
                    got.append(d.decode_frame(x[f]))
                    s1 = stats()
                    per.append([b - c for b, c in zip(s1, s0)])
                got = np.stack(got)
            else:
                got = d.decode_device(torch.from_numpy(x).cuda()).cpu().numpy()
            d.close()
        finally:
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        print(json.dumps({"path": label, "seg_stats_per_frame(ok,miss,noseg)": per, "diff": diff(got)}), flush=True)

    run("single-frame default (adaptive SEG)", {}, "frame")
    run("single-frame default again", {}, "frame")
    run("single-frame, plan warm-up only", {"VTB_SEG_ADAPT": "0"}, "frame")
    run("single-frame, SEG off (frame kernel)", {"VTB_DEBUG": "1024"}, "frame")
    run("single-frame, SEG off, no split", {"VTB_DEBUG": str(1024 | 256)}, "frame")
    run("batch decode_device", {}, "device")
    run("batch decode_device, no split", {"VTB_DEBUG": "256"}, "device")
    # round 4 bisection: the in-wave fix-up off (bit 14), forced on every split frame (bit 15),
    # forced and never converging (bits 15 + 16)
    run("single-frame, SEG off, no fix-up", {"VTB_DEBUG": str(1024 | 16384)}, "frame")
    run("batch decode_device, no fix-up", {"VTB_DEBUG": "16384"}, "device")
    run("batch decode_device, fix-up on every frame", {"VTB_DEBUG": "32768"}, "device")
    run("batch decode_device, fix-up never converging", {"VTB_DEBUG": str(32768 | 65536)}, "device")


if __name__ == "__main__":
    main()
