"""Golden node metrics of the reference's generic decoder for general-k codes
(tests/golden/genk_metrics.npz), produced by the reference itself: viterbiDecoderHard
(src/viterbiDecoder.c:52-234) compiled in place for the params/k4_k2n3 and params/k3_k3n4
configurations (oracle/_ref/librefgenk_*.so, oracle/Makefile) and driven with last=false
chunks of 7 segments, *nodeMetricsCur recorded after every chunk.  Inputs: payloads encoded
by the reference encoder, coded bits flipped with probability 0.06 (seeded numpy).

Run in the build container only:  make -C oracle ref && python tests/golden/make_golden_genk.py
"""
import ctypes
import hashlib
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_DIR = os.path.join(REPO, "oracle", "_ref")
CONFIGS = {"k4_k2n3": (2, 4, 3, 256), "k3_k3n4": (3, 3, 4, 192)}  # k, K, n, info bits
CHUNK = 7


def vp(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def main():
    out, sets = {}, {}
    seed = 4100
    for name, (k, K, n, L) in CONFIGS.items():
        enc = ctypes.CDLL(os.path.join(REF_DIR, f"librefenc_{name}.so"))
        gen = ctypes.CDLL(os.path.join(REF_DIR, f"librefgenk_{name}.so"))
        N = gen.refgenk_num_states()
        T = L // k + K - 1
        seed += 1
        rng = np.random.default_rng(seed)
        for f in range(4):
            unc = rng.integers(0, 256, L // 8, dtype=np.uint8)
            coded = np.zeros(T + 8, np.uint8)
            assert enc.refenc_encode(vp(unc), L // 8, vp(coded)) == T
            coded = coded[:T]
            flips = np.zeros(T, np.uint8)
            for i in range(n):
                flips |= (rng.random(T) < 0.06).astype(np.uint8) << i
            rx = np.ascontiguousarray(coded ^ flips)
            nch = (T + CHUNK - 1) // CHUNK
            met = np.zeros((nch, N), np.uint32)
            assert gen.refgenk_metrics(vp(rx), T, CHUNK, vp(met)) == nch
            out[f"{name}_f{f}_rx"] = rx
            out[f"{name}_f{f}_unc"] = unc
            out[f"{name}_f{f}_metrics"] = met
        sets[name] = {"k": k, "K": K, "n": n, "info_bits": L, "frames": 4, "p": 0.06, "chunk": CHUNK, "seed": seed,
                      "metric_bytes": gen.refgenk_metric_bytes()}
    path = os.path.join(HERE, "genk_metrics.npz")
    np.savez_compressed(path, **out)
    man_path = os.path.join(HERE, "MANIFEST.json")
    man = json.load(open(man_path))
    man["files"]["genk_metrics.npz"] = hashlib.sha256(open(path, "rb").read()).hexdigest()
    man.setdefault("sets", {})["genk_metrics"] = {"generator": "tests/golden/make_golden_genk.py", **sets}
    json.dump(man, open(man_path, "w"), indent=1, sort_keys=True)
    print("wrote", path, sets)


if __name__ == "__main__":
    main()
