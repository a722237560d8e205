"""Golden vectors for k = 1 codes with n != 2 (tests/golden/k1n.npz), produced by the
reference itself: oracle/_ref/libref_{k7n3,k9n3,k5n4,k8n3}.so are the reference's own
src/*.c compiled by oracle/Makefile with params/<name> (K and n compile-time, as the
reference's per-harness config directories).  Run in the build container only:

    make -C oracle && python tests/golden/make_golden_k1n.py

Every expected output is the reference's: convEnc for the error-free encoding,
viterbiDecoderHardButterflyk1 (last=true) for the decoded bytes, and nodeMetricsCur after
every 7-segment last=false chunk (ref_decode_stream).  Inputs are seeded numpy draws.
"""
import ctypes
import hashlib
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_DIR = os.path.join(REPO, "oracle", "_ref")

K1N = {"k7n3": (7, (0o133, 0o171, 0o165)), "k9n3": (9, (0o557, 0o663, 0o711)),
       "k5n4": (5, (0o23, 0o35, 0o27, 0o33)), "k8n3": (8, (0o225, 0o331, 0o367))}


def ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def load(name):
    K, g = K1N[name]
    lib = ctypes.CDLL(os.path.join(REF_DIR, f"libref_{name}.so"))
    vp, ci = ctypes.c_void_p, ctypes.c_int
    lib.ref_encode.argtypes = [vp, ci, vp]
    lib.ref_decode_frames.argtypes = [vp, ci, vp, ci, ci]
    lib.ref_decode_stream.argtypes = [vp, ci, ci, vp, vp]
    lib.ref_generator.restype = ctypes.c_ulong
    assert lib.ref_K() == K
    assert tuple(lib.ref_generator(i) for i in range(len(g))) == g
    return lib


def main():
    arrays, sets = {}, {}
    seed = 5000
    for name, (K, g) in K1N.items():
        lib = load(name)
        n, S = len(g), K - 1
        for L in (64, 1024):
            T = L + S
            F = 16 if L >= 1024 else 32
            for p in (0.0, 0.04, 0.1, 0.5):
                seed += 1
                rng = np.random.default_rng(seed)
                unc = rng.integers(0, 256, (F, L // 8), dtype=np.uint8)
                coded = np.zeros((F, T), np.uint8)
                for f in range(F):
                    row = np.ascontiguousarray(unc[f])
                    assert lib.ref_encode(ptr(row), L // 8, ptr(coded[f])) == T
                flips = np.zeros((F, T), np.uint8)
                for i in range(n):
                    flips |= (rng.random((F, T)) < p).astype(np.uint8) << i
                rx = coded ^ flips
                garbage = p == 0.04
                if garbage:  # the reference reads only the low n bits of each byte
                    rx = rx | (rng.integers(0, 256, (F, T), dtype=np.uint8) & np.uint8((0xFF << n) & 0xFF))
                rx = np.ascontiguousarray(rx, np.uint8)
                dec = np.zeros((F, L // 8), np.uint8)
                assert lib.ref_decode_frames(ptr(rx), T, ptr(dec), L // 8, F) == (L - 1) // 8 + 1
                key = f"{name}_L{L}_p{int(round(p * 1000)):03d}"
                arrays[key + "_uncoded"], arrays[key + "_rx"], arrays[key + "_decoded"] = unc, rx, dec
                sets[key] = {"seed": seed, "frames": F, "L": L, "p": p, "garbage_high_bits": garbage}
        # nodeMetricsCur after every 7-segment last=false chunk, then the last=true decode
        seed += 1
        rng = np.random.default_rng(seed)
        L, F, T = 256, 4, 256 + S
        for f in range(F):
            unc = rng.integers(0, 256, L // 8, dtype=np.uint8)
            coded = np.zeros(T, np.uint8)
            assert lib.ref_encode(ptr(unc), L // 8, ptr(coded)) == T
            flips = np.zeros(T, np.uint8)
            for i in range(n):
                flips |= (rng.random(T) < 0.08).astype(np.uint8) << i
            rx = np.ascontiguousarray(coded ^ flips, np.uint8)
            nch = (T + 6) // 7
            met = np.zeros((nch, 1 << S), np.uint8)
            out = np.zeros(L // 8, np.uint8)
            lib.ref_decode_stream(ptr(rx), T, 7, ptr(out), ptr(met))
            arrays[f"{name}_stream_f{f}_rx"] = rx
            arrays[f"{name}_stream_f{f}_metrics"] = met[: nch - 1]
            arrays[f"{name}_stream_f{f}_decoded"] = out
        sets[f"{name}_stream"] = {"seed": seed, "frames": F, "L": L, "p": 0.08, "chunk": 7}
    path = os.path.join(HERE, "k1n.npz")
    np.savez_compressed(path, **arrays)
    with open(path, "rb") as fh:
        digest = hashlib.sha256(fh.read()).hexdigest()
    man_path = os.path.join(HERE, "MANIFEST.json")
    with open(man_path) as fh:
        man = json.load(fh)
    man["files"]["k1n.npz"] = digest
    man.setdefault("sets", {})["k1n"] = {"generator": "tests/golden/make_golden_k1n.py",
                                         "codes": {k: [K, [oct(x) for x in g]] for k, (K, g) in K1N.items()},
                                         "sets": sets}
    with open(man_path, "w") as fh:
        json.dump(man, fh, indent=1, sort_keys=True)
    print("wrote", path, digest[:16])


if __name__ == "__main__":
    main()
