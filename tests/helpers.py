"""Test-side utilities: the oracle binding (test infrastructure only), golden fixtures and
seeded synthetic frames."""
import ctypes
import json
import os

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
ORACLE_LIB = os.path.join(REPO, "oracle", "build", "liboracle.so")
REF_DIR = os.path.join(REPO, "oracle", "_ref")

CODES = {5: (0o23, 0o35), 7: (0o113, 0o171), 9: (0o561, 0o753)}
BERTEST_P = (5.585640e-02, 3.716174e-02, 2.262231e-02)  # berTestK7.c:96
BERTEST_ERRORS = (92418, 9655, 655)  # reference run, SURVEY.md §4


def vp(a):
    return a.ctypes.data_as(ctypes.c_void_p)


class Oracle:
    """ctypes view of oracle/build/liboracle.so (the CPU restatement; checker only)."""

    def __init__(self, path=ORACLE_LIB):
        if not os.path.exists(path):
            import subprocess

            subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "oracle"], check=True, capture_output=True)
        L = ctypes.CDLL(path)
        v, i, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
        L.oracle_config_check.argtypes = [i, v]
        L.oracle_edge_table.argtypes = [i, v, v]
        L.oracle_encode.argtypes = [i, v, v, i, v]
        L.oracle_genk_encode.argtypes = [i, i, i, v, v, i, v]
        L.oracle_genk_decode.argtypes = [i, i, i, v, v, i, v]
        L.oracle_genk_metrics.argtypes = [i, i, i, v, v, i, v, v]
        L.oracle_k1n_decode.argtypes = [i, i, v, v, i, v]
        L.oracle_decode_hard.argtypes = [i, v, v, i, v]
        L.oracle_decode_soft.argtypes = [i, v, v, i, v]
        L.oracle_decode_batch.argtypes = [i, v, i, v, sz, i, v, sz, sz, i]
        L.oracle_stream_create.restype = v
        L.oracle_stream_create.argtypes = [i, v]
        L.oracle_stream_destroy.argtypes = [v]
        L.oracle_stream_decode.argtypes = [v, v, i, v, i, v]
        L.oracle_bertest_stream.restype = ctypes.c_long
        L.oracle_bertest_stream.argtypes = [i, v, ctypes.c_uint, i, v, i, i, v, v]
        u64 = ctypes.c_uint64
        L.oracle_rand64.restype = u64
        L.oracle_rand64.argtypes = [u64, u64, u64]
        L.oracle_gen_payload.argtypes = [u64, i, v, sz, sz]
        L.oracle_gen_encode.argtypes = [i, v, i, v, sz, v, sz, sz]
        L.oracle_gen_bsc.argtypes = [u64, ctypes.c_uint32, i, v, sz, v, sz, sz]
        L.oracle_gen_awgn8.argtypes = [u64, ctypes.c_int64, i, v, sz, v, sz, sz]
        L.oracle_awgn_kq.restype = ctypes.c_int64
        L.oracle_awgn_kq.argtypes = [ctypes.c_double]
        L.oracle_bsc_p32.restype = ctypes.c_uint32
        L.oracle_bsc_p32.argtypes = [ctypes.c_double]
        self.L = L

    # -- device frame generator checker (include/viterbi_amd.h "Synthetic frames") --
    def rand64(self, seed, frame, ctr):
        return int(self.L.oracle_rand64(seed, frame, ctr))

    def gen_payload(self, seed, bits, frames):
        nb = (bits + 7) // 8
        out = np.zeros((frames, nb), np.uint8)
        self.L.oracle_gen_payload(seed, bits, vp(out), nb, frames)
        return out

    def gen_encode(self, K, g, bits, unc):
        unc = np.ascontiguousarray(unc, np.uint8)
        T = bits + K - 1
        out = np.zeros((unc.shape[0], T), np.uint8)
        self.L.oracle_gen_encode(K, self._g(g), bits, vp(unc), unc.shape[1], vp(out), T, unc.shape[0])
        return out

    def gen_bsc(self, seed, p32, coded):
        coded = np.ascontiguousarray(coded, np.uint8)
        F, T = coded.shape
        out = np.zeros((F, T), np.uint8)
        self.L.oracle_gen_bsc(seed, p32, T, vp(coded), T, vp(out), T, F)
        return out

    def gen_awgn8(self, seed, kq, coded):
        coded = np.ascontiguousarray(coded, np.uint8)
        F, T = coded.shape
        out = np.zeros((F, T, 2), np.uint8)
        self.L.oracle_gen_awgn8(seed, kq, T, vp(coded), T, vp(out), 2 * T, F)
        return out

    @staticmethod
    def _g(g):
        return (ctypes.c_uint64 * 2)(*g)

    def config_check(self, K, g):
        return self.L.oracle_config_check(K, self._g(g))

    def edge_table(self, K, g):
        out = np.zeros(1 << (K - 2), np.uint8)
        self.L.oracle_edge_table(K, self._g(g), vp(out))
        return out

    def encode(self, K, g, uncoded):
        unc = np.ascontiguousarray(uncoded, np.uint8)
        F, nb = unc.shape
        T = 8 * nb + K - 1
        out = np.zeros((F, T), np.uint8)
        G = self._g(g)
        for f in range(F):
            row = np.ascontiguousarray(unc[f])
            o = np.zeros(T, np.uint8)
            assert self.L.oracle_encode(K, G, vp(row), nb, vp(o)) == T
            out[f] = o
        return out

    def genk_encode(self, k, K, g, uncoded):
        """Rows of payload bytes -> rows of info_bits/k + K-1 coded segments (oracle_genk_encode)."""
        unc = np.ascontiguousarray(uncoded, np.uint8)
        F, nb = unc.shape
        T = 8 * nb // k + K - 1
        G = (ctypes.c_uint64 * 8)(*[int(v) for v in g])
        out = np.zeros((F, T), np.uint8)
        for f in range(F):
            row = np.ascontiguousarray(unc[f])
            o = np.zeros(T, np.uint8)
            assert self.L.oracle_genk_encode(k, K, len(g), G, vp(row), nb, vp(o)) == T
            out[f] = o
        return out

    def genk_decode(self, k, K, g, frames, info_bits):
        x = np.ascontiguousarray(frames, np.uint8)
        G = (ctypes.c_uint64 * 8)(*[int(v) for v in g])
        nb = (info_bits + 7) // 8
        out = np.zeros((x.shape[0], nb), np.uint8)
        for f in range(x.shape[0]):
            row = np.ascontiguousarray(x[f])
            o = np.zeros(nb, np.uint8)
            assert self.L.oracle_genk_decode(k, K, len(g), G, vp(row), info_bits, vp(o)) == nb
            out[f] = o
        return out

    def k1n_decode(self, K, g, frames, info_bits):
        """The reference k=1 decoder for any n (oracle_k1n_decode: uint8 butterfly arithmetic)."""
        x = np.ascontiguousarray(frames, np.uint8)
        G = (ctypes.c_uint64 * 8)(*[int(v) for v in g])
        nb = (info_bits + 7) // 8
        out = np.zeros((x.shape[0], nb), np.uint8)
        for f in range(x.shape[0]):
            row = np.ascontiguousarray(x[f])
            o = np.zeros(nb, np.uint8)
            assert self.L.oracle_k1n_decode(K, len(g), G, vp(row), info_bits, vp(o)) == nb
            out[f] = o
        return out

    def genk_metrics(self, k, K, g, coded, metrics):
        """The generic decoder's metric update (oracle_genk_metrics): (metrics, prev)."""
        m = np.ascontiguousarray(metrics, np.uint32).copy()
        prev = np.zeros_like(m)
        G = (ctypes.c_uint64 * 8)(*[int(v) for v in g])
        row = np.ascontiguousarray(coded, np.uint8)
        assert self.L.oracle_genk_metrics(k, K, len(g), G, vp(row), len(row), vp(m), vp(prev)) == 0
        return m, prev

    def decode(self, K, g, frames, L, soft=False, threads=8):
        x = np.ascontiguousarray(frames, np.uint8)
        F = x.shape[0]
        x = x.reshape(F, -1)
        T = L + K - 1
        assert x.shape[1] == (2 * T if soft else T)
        ob = (L + 7) // 8
        out = np.zeros((F, ob), np.uint8)
        rc = self.L.oracle_decode_batch(K, self._g(g), int(soft), vp(x), x.shape[1], T, vp(out), ob, F, threads)
        assert rc == 0
        return out

    def stream(self, K, g):
        return OracleStream(self, K, g)

    def bertest(self, K=7, g=CODES[7], seed=9865, p=BERTEST_P, npkts=10000, pkt_bytes=256):
        T = 8 * pkt_bytes + K - 1
        unc = np.zeros((len(p), npkts, pkt_bytes), np.uint8)
        rx = np.zeros((len(p), npkts, T), np.uint8)
        pa = (ctypes.c_double * len(p))(*p)
        flips = self.L.oracle_bertest_stream(K, self._g(g), seed, len(p), pa, npkts, pkt_bytes, vp(unc), vp(rx))
        return unc, rx, flips


class OracleStream:
    def __init__(self, orc, K, g):
        self.orc, self.K, self.N = orc, K, 1 << (K - 1)
        self.h = orc.L.oracle_stream_create(K, orc._g(g))

    def decode(self, coded, out, last):
        c = np.ascontiguousarray(coded, np.uint8)
        met = np.zeros(self.N, np.uint8)
        r = self.orc.L.oracle_stream_decode(self.h, vp(c), len(c), vp(out), int(last), vp(met))
        return r, met

    def __del__(self):
        try:
            self.orc.L.oracle_stream_destroy(self.h)
        except Exception:
            pass


def load_golden(name):
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def manifest():
    with open(os.path.join(GOLDEN, "MANIFEST.json")) as fh:
        return json.load(fh)


def golden_sets(K):
    """Yield (key, L, uncoded, rx, decoded) for every hard set of constraint length K."""
    z = load_golden(f"k{K}_hard.npz")
    keys = sorted({k.rsplit("_", 1)[0] for k in z})
    for key in keys:
        L = int(key.split("_")[0][1:])
        yield key, L, z[key + "_uncoded"], z[key + "_rx"], z[key + "_decoded"]


# tests/golden/lengths.npz (make_golden_lengths.py): reference-decoded frames of every k = 1 rate-1/2
# constraint length the legacy drop-in builds (params/<name>, oracle/_ref/libref_<name>.so) at
# L in LENGTHS, BSC p in {0.03, 0.5}.  "k3" is handTraced's non-symmetric code.
LENGTH_CODES = {"k3": (3, (0b111, 0b110)), "k3s": (3, (0o7, 0o5)), "k4": (4, (0o15, 0o17)), "k5": (5, (0o23, 0o35)),
                "k6": (6, (0o53, 0o75)), "k7": (7, (0o113, 0o171)), "k8": (8, (0o247, 0o371)),
                "k9": (9, (0o561, 0o753))}
LENGTHS = (1, 7, 100, 1001, 4095, 9000, 16383, 16384)


def length_sets(names=None, lengths=None):
    """Yield (key, name, K, g, L, uncoded, rx, decoded) from tests/golden/lengths.npz."""
    z = load_golden("lengths.npz")
    sets = manifest()["lengths"]["sets"]
    for key in sorted(sets, key=lambda k: (k.split("_")[0], sets[k]["L"], sets[k]["p"])):
        name = key.split("_")[0]
        info = sets[key]
        if (names is not None and name not in names) or (lengths is not None and info["L"] not in lengths):
            continue
        yield (key, name, info["K"], tuple(info["g"]), info["L"], z[key + "_uncoded"], z[key + "_rx"],
               z[key + "_decoded"])


def random_frames(orc, K, L, frames, p, seed, soft=False, sigma=None, g=None):
    """Seeded terminated frames through a BSC (hard) or BPSK-AWGN + 8-bit quantiser (soft).

    Soft quantiser: y = (1-2b) + sigma*noise, q = clamp(round((1-y)/2*255)).
    Returns (uncoded_bytes [F, ceil(L/8)], rx [F, T] or [F, T, 2])."""
    rng = np.random.default_rng(seed)
    nb = (L + 7) // 8
    unc = rng.integers(0, 256, (frames, nb), dtype=np.uint8)
    if L % 8:
        unc[:, -1] &= np.uint8((0xFF << (8 - L % 8)) & 0xFF)
    bits = np.unpackbits(unc, axis=1)[:, :L]
    coded = encode_bits(K, g if g is not None else CODES[K], bits, orc)
    T = L + K - 1
    if not soft:
        flips = (rng.random((frames, T, 2)) < p).astype(np.uint8)
        return unc, (coded ^ (flips[..., 0] | (flips[..., 1] << 1))).astype(np.uint8)
    b = np.stack([coded & 1, (coded >> 1) & 1], axis=-1).astype(np.float64)
    y = (1.0 - 2.0 * b) + (sigma if sigma is not None else 0.5) * rng.standard_normal(b.shape)
    q = np.clip(np.rint((1.0 - y) * 0.5 * 255.0), 0, 255).astype(np.uint8)
    return unc, q


def encode_bits(K, g, bits, orc=None):
    """Terminated encoding of arbitrary-length bit rows (vectorised restatement of
    convEncode.c:46-130; whole-byte rows are cross-checked against the oracle encoder)."""
    bits = np.asarray(bits, np.uint8)
    F, L = bits.shape
    S = K - 1
    padded = np.concatenate([np.zeros((F, S), np.uint8), bits, np.zeros((F, S), np.uint8)], axis=1)
    T = L + S
    # tapped-delay bit i (i steps ago) at step t is padded[:, t + S - i]
    revs = []
    for gi in g:
        rv = [(gi >> (K - 1 - i)) & 1 for i in range(K)]  # reversed: bit i of poly = MSB-i of g
        revs.append(rv)
    out = np.zeros((F, T), np.uint8)
    for j, rv in enumerate(revs):
        acc = np.zeros((F, T), np.uint8)
        for i in range(K):
            if rv[i]:
                acc ^= padded[:, S - i:S - i + T]
        out |= (acc << j).astype(np.uint8)
    return out


def hard_to_soft(rx):
    """Map hard segments to the soft format's hard-equivalent input q = 255*bit."""
    rx = np.asarray(rx, np.uint8)
    return np.stack([(rx & 1) * 255, ((rx >> 1) & 1) * 255], axis=-1).astype(np.uint8)


# General rate-k/n codes (k, K, generators over k*K bits) for the general-k decoder
# (SURVEY.md 8 f4).  The first two are params/k4_k2n3 and params/k3_k3n4, whose reference
# encoder oracle/Makefile builds (oracle/_ref/librefenc_*.so).
GENK_CODES = (
    (2, 4, (0xB5, 0x6B, 0xD9)),
    (3, 3, (0x1ED, 0x15B, 0x0B7, 0x1A7)),
    (4, 3, (0xB5D, 0x6E3, 0x9A7, 0xF19, 0x5CB)),
    (2, 5, (0x2DB, 0x1B5, 0x3A7)),
    (1, 7, (0o113, 0o171)),
    (2, 3, (0x2B, 0x1D, 0x37)),
)
GENK_REF_PARAMS = {"k4_k2n3": GENK_CODES[0], "k3_k3n4": GENK_CODES[1]}

# k = 1 codes with n != 2 (params/k7n3, k9n3, k5n4, k8n3): the reference decoder is generic in n
# (viterbiDecoderButterflyk1.c:104-107); oracle/_ref/libref_<name>.so is the reference built
# with each, tests/golden/k1n.npz its outputs.
K1N_PARAMS = {"k7n3": (7, (0o133, 0o171, 0o165)), "k9n3": (9, (0o557, 0o663, 0o711)),
              "k5n4": (5, (0o23, 0o35, 0o27, 0o33)), "k8n3": (8, (0o225, 0o331, 0o367))}


def k1n_frames(orc, K, g, L, F, p, seed, garbage=False):
    """Random payloads encoded with an n-generator k=1 code (oracle_genk_encode with k = 1),
    each coded bit flipped with probability p; garbage=True sets the unused high bits of every
    segment byte (the reference reads only the low n bits, viterbiDecoder.c:278-281)."""
    unc, rx = genk_frames(orc, 1, K, g, L, F, p, seed)
    if garbage:
        rng = np.random.default_rng(seed + 1)
        n = len(g)
        rx = rx | (rng.integers(0, 256, rx.shape, dtype=np.uint8) & np.uint8((0xFF << n) & 0xFF))
    return unc, rx.astype(np.uint8)


def legacy_layout(k, K, n):
    """Byte offsets of viterbiHardState_t (include/viterbiDecoder.h, the reference's
    src/viterbiDecoder.h:103-146 layout) for a code configuration, as the C compiler lays
    it out (tests/test_legacy_abi.py checks this against a compiled probe)."""
    N, E = 1 << (k * (K - 1)), 1 << k
    if k == 1:
        mb = 1
    else:
        span = n * (16 * 1024 + K - 1)
        mb = 1 if span <= 1 << 8 else 2 if span <= 1 << 16 else 4

    def align(x, a):
        return (x + a - 1) // a * a

    off = N // 2 + E * N  # edgeCodedBitsSymm, edgeCodedBits (uint8)
    lay = {"N": N, "metric_bytes": mb}
    lay["nodeMetricsA"] = off = align(off, 64)
    lay["traceBackA"] = off = align(off + N * mb, 64)
    lay["nodeMetricsB"] = off = align(off + N, mb)
    lay["traceBackB"] = off = off + N * mb
    lay["nodeMetricsCur"] = off = align(off + N, 8)
    lay["traceBackCur"], lay["nodeMetricsNext"], lay["traceBackNext"] = off + 8, off + 16, off + 24
    lay["iteration"] = off + 32
    lay["renormCounter"] = off + 36
    lay["decodeCarryOverCount"] = off + 41
    lay["tracebackBufs"] = off = align(off + 42, 64)
    lay["sizeof"] = align(off + (16 * 1024 + (K - 1) * k) * N, 64)
    return lay


def genk_frames(orc, k, K, g, info_bits, F, p, seed):
    """Random payloads, encoded by the oracle, each coded bit flipped with probability p."""
    rng = np.random.default_rng(seed)
    unc = rng.integers(0, 256, (F, info_bits // 8), dtype=np.uint8)
    coded = orc.genk_encode(k, K, g, unc)
    n = len(g)
    flips = np.zeros(coded.shape, np.uint8)
    for i in range(n):
        flips |= ((rng.random(coded.shape) < p).astype(np.uint8) << i)
    return unc, coded ^ flips
