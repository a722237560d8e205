"""The reference's speedDecode protocol (16 packets of 2,048 bits, srand(314), one frame per
VITERBI_DECODER_HARD call with last=true; speedDecode/speedDecode.c:37-116) through the legacy
drop-in of every k = 1 rate-1/2 configuration, beside the reference decoder compiled with the
same configuration (oracle/_ref/libref_<name>.so) on one host core.  Measurement only.

    python tools/legacy_speed.py [--seconds S] [--names k3s,k4,k5,k6,k7,k8,k9]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))

from helpers import LENGTH_CODES, encode_bits, legacy_layout  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=2.0)
    ap.add_argument("--names", default="k3s,k4,k5,k6,k7,k8,k9")
    args = ap.parse_args()
    lib_dir = os.path.join(REPO, "convolutionalencdec_amd", "lib")
    for name in args.names.split(","):
        K, g = LENGTH_CODES[name]
        rng = np.random.default_rng(314)
        unc = rng.integers(0, 256, (16, 256), dtype=np.uint8)
        coded = np.ascontiguousarray(encode_bits(K, g, np.unpackbits(unc, axis=1)))
        T = coded.shape[1]
        lib = ctypes.CDLL(os.path.join(lib_dir, f"libviterbi_legacy_{name}.so"))
        v = ctypes.c_void_p
        lib.viterbiInitButterflyk1.argtypes = [v]
        lib.resetViterbiDecoderHardButterflyk1.argtypes = [v]
        lib.viterbiDecoderHardButterflyk1.argtypes = [v, v, v, ctypes.c_int, ctypes.c_bool]
        buf = np.zeros(legacy_layout(1, K, 2)["sizeof"] + 64, np.uint8)
        st = ctypes.c_void_p(buf.ctypes.data + (-buf.ctypes.data) % 64)
        lib.resetViterbiDecoderHardButterflyk1(st)
        lib.viterbiInitButterflyk1(st)
        out = np.zeros(256, np.uint8)
        rows = [ctypes.c_void_p(coded[i].ctypes.data) for i in range(16)]
        op = ctypes.c_void_p(out.ctypes.data)
        for i in range(32):  # warm-up (plan, code objects)
            lib.viterbiDecoderHardButterflyk1(st, rows[i % 16], op, T, True)
        n, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < args.seconds:
            for i in range(16):
                lib.viterbiDecoderHardButterflyk1(st, rows[i], op, T, True)
            n += 16
        gpu = n * 2048 / (time.perf_counter() - t0) / 1e6
        assert (out == unc[(n - 1) % 16]).all()
        ref = ctypes.CDLL(os.path.join(REPO, "oracle", "_ref", f"libref_{name}.so"))
        ref.ref_speed.restype = ctypes.c_double
        ref.ref_speed.argtypes = [ctypes.c_double, ctypes.c_int, ctypes.c_int]
        cpu = ref.ref_speed(args.seconds, 1, 256)
        print(json.dumps({"config": name, "K": K, "dropin_mbps": round(gpu, 1), "reference_1core_mbps": round(cpu, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
