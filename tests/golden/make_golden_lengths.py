"""Reference-decoded frames at every frame length the GPU tests use.

Run in the build container only (needs oracle/_ref/libref_*.so, which oracle/Makefile compiles
from /root/reference/src with one code-parameter directory each):

    make -C oracle && python tests/golden/make_golden_lengths.py

Writes tests/golden/lengths.npz and its entry in MANIFEST.json ("files", "lengths").

Every expected output is the reference decoder's (viterbiDecoderHardButterflyk1 through
ref_decode_frames, /root/reference/src/viterbiDecoderButterflyk1.c:82-263), called with the
whole frame and last=true, as the reference harnesses do.  The reference decoder takes any
segment count: a frame of L information bits that is not a whole number of bytes gets its
partial last byte zeroed and filled MSB-first (:226-227, 243-249).  Only the reference
encoder needs whole bytes (convEnc, src/convEncode.c:46-130), so the inputs are encoded here
bit by bit (a vectorised restatement of the same shift register, helpers.encode_bits) and
cross-checked against the reference encoder wherever L is a multiple of 8.  Inputs are seeded
numpy draws; encoding is input preparation only -- nothing in the expected output comes from
this repository's oracle or product.

Codes (the legacy drop-in builds a library for each: Makefile LEGACY_KS):
  k3   handTraced's K=3 (0b111, 0b110): g[1] lacks the newest-input tap, so the reference's
       butterfly applies its n - e complement to a code it does not fit (VERDICT r5 missing #4)
  k3s  K=3 (07, 05); k4 (015, 017); k5 (023, 035); k6 (053, 075); k7 (0113, 0171, the
       reference's default); k8 (0247, 0371); k9 (0561, 0753)
"""
import ctypes
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_DIR = os.path.join(REPO, "oracle", "_ref")
sys.path.insert(0, os.path.dirname(HERE))

from helpers import encode_bits  # noqa: E402

CODES = {"k3": (3, (0b111, 0b110)), "k3s": (3, (0o7, 0o5)), "k4": (4, (0o15, 0o17)), "k5": (5, (0o23, 0o35)),
         "k6": (6, (0o53, 0o75)), "k7": (7, (0o113, 0o171)), "k8": (8, (0o247, 0o371)), "k9": (9, (0o561, 0o753))}
LENGTHS = (1, 7, 100, 1001, 4095, 9000, 16383, 16384)
PS = (0.03, 0.5)


def frames_for(L):
    return 8 if L <= 1001 else 2


def load_ref(name):
    K, g = CODES[name]
    lib = ctypes.CDLL(os.path.join(REF_DIR, f"libref_{name}.so"))
    vp, ci = ctypes.c_void_p, ctypes.c_int
    lib.ref_encode.argtypes = [vp, ci, vp]
    lib.ref_decode_frames.argtypes = [vp, ci, vp, ci, ci]
    lib.ref_generator.restype = ctypes.c_ulong
    assert lib.ref_K() == K and (lib.ref_generator(0), lib.ref_generator(1)) == g, name
    assert lib.ref_max_segments() == 16384 + K - 1
    return lib


def ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def main():
    arrays, sets = {}, {}
    seed = 60000
    for name, (K, g) in CODES.items():
        lib = load_ref(name)
        for L in LENGTHS:
            F = frames_for(L)
            T = L + K - 1
            for p in PS:
                seed += 1
                rng = np.random.default_rng(seed)
                unc = rng.integers(0, 256, (F, (L + 7) // 8), dtype=np.uint8)
                if L % 8:
                    unc[:, -1] &= np.uint8((0xFF << (8 - L % 8)) & 0xFF)
                coded = encode_bits(K, g, np.unpackbits(unc, axis=1)[:, :L])
                if L % 8 == 0:  # the reference encoder agrees wherever it applies
                    for f in range(F):
                        o = np.zeros(T, np.uint8)
                        row = np.ascontiguousarray(unc[f])
                        assert lib.ref_encode(ptr(row), L // 8, ptr(o)) == T
                        assert (o == coded[f]).all(), (name, L, f)
                flips = (rng.random((F, T, 2)) < p).astype(np.uint8)
                rx = np.ascontiguousarray(coded ^ (flips[..., 0] | (flips[..., 1] << 1)), np.uint8)
                dec = np.zeros((F, (L + 7) // 8), np.uint8)
                r = lib.ref_decode_frames(ptr(rx), T, ptr(dec), dec.shape[1], F)
                assert r == (L - 1) // 8 + 1, (name, L, r)
                key = f"{name}_L{L}_p{int(round(p * 1000)):03d}"
                arrays[key + "_uncoded"] = unc
                arrays[key + "_rx"] = rx
                arrays[key + "_decoded"] = dec
                sets[key] = {"K": K, "g": [int(x) for x in g], "L": L, "p": p, "frames": F, "seed": seed}
    path = os.path.join(HERE, "lengths.npz")
    np.savez_compressed(path, **arrays)
    with open(os.path.join(HERE, "MANIFEST.json")) as fh:
        manifest = json.load(fh)
    with open(path, "rb") as fh:
        manifest["files"]["lengths.npz"] = hashlib.sha256(fh.read()).hexdigest()
    manifest["lengths"] = {"generator": "tests/golden/make_golden_lengths.py", "codes": {k: [v[0], list(v[1])]
                           for k, v in CODES.items()}, "sets": sets}
    with open(os.path.join(HERE, "MANIFEST.json"), "w") as fh:
        json.dump(manifest, fh, indent=1, sort_keys=True)
    print("wrote lengths.npz:", len(sets), "sets,", os.path.getsize(path), "bytes")


if __name__ == "__main__":
    sys.exit(main())
