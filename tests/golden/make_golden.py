"""Generate the golden vectors in tests/golden/ from the reference itself.

Run in the build container only (needs oracle/_ref/libref_k*.so, which oracle/Makefile
compiles from /root/reference/src):

    make -C oracle && python tests/golden/make_golden.py

Every expected output here is produced by the reference decoder / encoder
(viterbiDecoderHardButterflyk1, convEnc) -- never by this repo's oracle or product.
Inputs are seeded numpy draws (seeds recorded in MANIFEST.json).  The soft "bridge"
fixture maps each hard frame to 8-bit soft input q = 255*bit; its expected output is the
reference's hard decode of the same frame ("Soft-decision format").
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

CODES = {3: (0b111, 0b110), 5: (0o23, 0o35), 7: (0o113, 0o171), 9: (0o561, 0o753)}


def load_ref(K):
    lib = ctypes.CDLL(os.path.join(REF_DIR, f"libref_k{K}.so"))
    vp, ci = ctypes.c_void_p, ctypes.c_int
    lib.ref_encode.argtypes = [vp, ci, vp]
    lib.ref_decode_frames.argtypes = [vp, ci, vp, ci, ci]
    lib.ref_decode_stream.argtypes = [vp, ci, ci, vp, vp]
    lib.ref_edge_table.argtypes = [vp]
    lib.ref_state_size.restype = ctypes.c_ulong
    lib.ref_generator.restype = ctypes.c_ulong
    assert lib.ref_K() == K
    assert (lib.ref_generator(0), lib.ref_generator(1)) == CODES[K]
    return lib


def ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def encode(lib, unc, T):
    F, nb = unc.shape
    coded = np.zeros((F, T), np.uint8)
    for f in range(F):
        row = np.ascontiguousarray(unc[f])
        out = np.zeros(T, np.uint8)
        assert lib.ref_encode(ptr(row), nb, ptr(out)) == T
        coded[f] = out
    return coded


def decode(lib, coded, L):
    F, T = coded.shape
    out = np.zeros((F, (L + 7) // 8), np.uint8)
    c = np.ascontiguousarray(coded)
    r = lib.ref_decode_frames(ptr(c), T, ptr(out), out.shape[1], F)
    assert r == (L - 1) // 8 + 1, r
    return out


def noisy_set(lib, K, L, p, frames, seed, garbage):
    rng = np.random.default_rng(seed)
    S = K - 1
    T = L + S
    unc = rng.integers(0, 256, (frames, (L + 7) // 8), dtype=np.uint8)
    if L % 8:
        unc[:, -1] &= np.uint8((0xFF << (8 - L % 8)) & 0xFF)
    if L % 8 == 0:
        coded = encode(lib, unc, T)
    else:  # convEnc only takes whole bytes: encode bit-exactly via a padded copy is not
        raise ValueError("L must be a multiple of 8 for the reference encoder")
    flips = (rng.random((frames, T, 2)) < p).astype(np.uint8)
    rx = coded ^ (flips[..., 0] | (flips[..., 1] << 1))
    if garbage:  # the reference reads only the low n bits of each segment byte
        rx = rx | (rng.integers(0, 64, (frames, T), dtype=np.uint8) << 2)
    dec = decode(lib, rx, L)
    return unc, rx.astype(np.uint8), dec


def main():
    manifest = {"generator": "tests/golden/make_golden.py", "reference": "/root/reference (v1.0.1)",
                "files": {}}
    written = []

    def save(name, **arrays):
        path = os.path.join(HERE, name)
        np.savez_compressed(path, **arrays)
        written.append(name)

    tables = {}
    sizes = {}
    for K in (3, 5, 7, 9):
        lib = load_ref(K)
        e = np.zeros(1 << (K - 2), np.uint8)
        lib.ref_edge_table(ptr(e))
        tables[f"k{K}"] = e
        sizes[K] = int(lib.ref_state_size())
    save("edge_tables.npz", **tables)

    # handTraced.c:29-47 encoder KAT (K=3, g={0b111, 0b110}), reproduced through the reference
    lib3 = load_ref(3)
    enc_kat = encode(lib3, np.array([[0b01101000]], np.uint8), 8 + 2)[0]
    assert list(enc_kat) == [0, 3, 0, 2, 2, 3, 1, 0, 0, 0], list(enc_kat)

    seed = 1000
    sets = {}
    for K, Ls, ps in ((7, (8, 64, 1024, 2048), (0.0, 0.03, 0.06, 0.5)),
                      (9, (64, 1024), (0.0, 0.03, 0.06, 0.5)),
                      (5, (1024,), (0.0, 0.06, 0.5))):
        lib = load_ref(K)
        arrays = {}
        for L in Ls:
            frames = 32 if L >= 1024 else 64
            for p in ps:
                seed += 1
                unc, rx, dec = noisy_set(lib, K, L, p, frames, seed, garbage=(p == 0.06))
                key = f"L{L}_p{int(round(p * 1000)):03d}"
                arrays[key + "_uncoded"] = unc
                arrays[key + "_rx"] = rx
                arrays[key + "_decoded"] = dec
                sets[f"k{K}/{key}"] = {"seed": seed, "frames": frames, "L": L, "p": p,
                                       "garbage_high_bits": p == 0.06}
        save(f"k{K}_hard.npz", **arrays)

    # Streaming: nodeMetricsCur after each 7-segment chunk (last=false), K=7 and K=9.
    stream = {}
    for K in (7, 9):
        lib = load_ref(K)
        seed += 1
        unc, rx, dec = noisy_set(lib, K, 256, 0.06, 4, seed, garbage=False)
        T = rx.shape[1]
        chunk = 7
        nchunks = (T + chunk - 1) // chunk
        for f in range(rx.shape[0]):
            met = np.zeros((nchunks, 1 << (K - 1)), np.uint8)
            out = np.zeros(32, np.uint8)
            row = np.ascontiguousarray(rx[f])
            lib.ref_decode_stream(ptr(row), T, chunk, ptr(out), ptr(met))
            assert (out == dec[f]).all()
            stream[f"k{K}_f{f}_rx"] = row
            stream[f"k{K}_f{f}_metrics"] = met[: nchunks - 1]
            stream[f"k{K}_f{f}_decoded"] = out
        sets[f"stream/k{K}"] = {"seed": seed, "frames": 4, "L": 256, "p": 0.06, "chunk": chunk}
    save("stream_metrics.npz", **stream)

    manifest["sets"] = sets
    manifest["kat"] = {
        "handTraced_encoder_K3": {"uncoded": [0x68], "coded": [int(x) for x in enc_kat],
                                  "source": "handTracedTest/handTraced.c:29-47"},
        "berTestK7_decoded_bit_errors": {"seed": 9865, "packets": 10000, "packet_bytes": 256,
                                         "p": [5.585640e-02, 3.716174e-02, 2.262231e-02],
                                         "errors": [92418, 9655, 655], "bits_per_config": 20480000,
                                         "source": "berTestK7/berTestK7.c:55-172, measured by "
                                                   "running the reference harness (SURVEY.md §4)"},
        "viterbiHardState_t_sizeof": {str(K): v for K, v in sizes.items()},
        "k7_edge_table": [int(x) for x in tables["k7"]],
    }
    for name in written:
        with open(os.path.join(HERE, name), "rb") as fh:
            manifest["files"][name] = hashlib.sha256(fh.read()).hexdigest()
    with open(os.path.join(HERE, "MANIFEST.json"), "w") as fh:
        json.dump(manifest, fh, indent=1, sort_keys=True)
    print("wrote", written)


if __name__ == "__main__":
    sys.exit(main())
