"""The legacy C API's per-call semantics on the GPU (include/viterbiDecoder.h through
libviterbi_legacy_<config>.so):

* nodeMetricsCur (and renormCounter) after every last=false chunk equal the reference's
  (viterbiDecoderButterflyk1.c:101-191, golden tests/golden/stream_metrics.npz produced by
  the reference; k>1: viterbiDecoder.c:84-131, golden tests/golden/genk_metrics.npz);
* VITERBI_DECODER_HARD for k>1 (viterbiDecoderHard) decodes whole frames on the GPU,
  checked against the oracle's terminated ML decode (the reference's own k>1 traceback is
  broken);
* vtb_legacy_metrics_k1 against the oracle's uint8 streaming restatement for random
  chunkings, including the reference's non-symmetric K=3 handTraced code.
"""
import ctypes
import os

import numpy as np
import pytest

from helpers import CODES, GENK_REF_PARAMS, Oracle, genk_frames, legacy_layout, load_golden, random_frames, vp

pytestmark = pytest.mark.gpu

CONFIGS = {"k7": (1, 7, 2), "k9": (1, 9, 2), "k4_k2n3": (2, 4, 3), "k3_k3n4": (3, 3, 4),
           "k7n3": (1, 7, 3), "k9n3": (1, 9, 3), "k5n4": (1, 5, 4), "k8n3": (1, 8, 3)}


@pytest.fixture(scope="module")
def orc():
    return Oracle()


class Legacy:
    """One legacy library and a caller-allocated state struct (numpy buffer, 64-B aligned)."""

    def __init__(self, name):
        from convolutionalencdec_amd import LIB_DIR

        self.k, self.K, self.n = CONFIGS[name]
        self.lay = legacy_layout(self.k, self.K, self.n)
        L = ctypes.CDLL(os.path.join(LIB_DIR, f"libviterbi_legacy_{name}.so"))
        v = ctypes.c_void_p
        for f in ("viterbiInitButterflyk1", "resetViterbiDecoderHardButterflyk1", "viterbiInit", "resetViterbiDecoderHard"):
            getattr(L, f).argtypes = [v]
        for f in ("viterbiDecoderHardButterflyk1", "viterbiDecoderHard"):
            getattr(L, f).argtypes = [v, v, v, ctypes.c_int, ctypes.c_bool]
        self.L = L
        self.buf = np.zeros(self.lay["sizeof"] + 64, np.uint8)
        self.off = (-self.buf.ctypes.data) % 64
        self.st = ctypes.c_void_p(self.buf.ctypes.data + self.off)
        if self.k == 1:
            L.resetViterbiDecoderHardButterflyk1(self.st)
            L.viterbiInitButterflyk1(self.st)
            self.dec = L.viterbiDecoderHardButterflyk1
        else:
            L.resetViterbiDecoderHard(self.st)
            L.viterbiInit(self.st)
            self.dec = L.viterbiDecoderHard

    def call(self, seg, out, last):
        seg = np.ascontiguousarray(seg, np.uint8)
        return self.dec(self.st, vp(seg), vp(out), len(seg), bool(last))

    def _field(self, name, dtype, count=1):
        o = self.off + self.lay[name]
        return np.frombuffer(self.buf[o:o + np.dtype(dtype).itemsize * count].tobytes(), dtype)

    def metrics_cur(self):
        """*nodeMetricsCur: the pointer in the struct, dereferenced into the buffer."""
        p = int(self._field("nodeMetricsCur", np.uint64)[0]) - self.buf.ctypes.data
        mb = self.lay["metric_bytes"]
        return np.frombuffer(self.buf[p:p + mb * self.lay["N"]].tobytes(), {1: np.uint8, 2: np.uint16, 4: np.uint32}[mb])

    def renorm_counter(self):
        return int(self._field("renormCounter", np.uint32)[0])

    def iteration(self):
        return int(self._field("iteration", np.uint32)[0])


def _renorm_phase(t):
    """The reference's renormCounter after t steps (:159-183: fires at 120, 241, ...)."""
    c = 0
    for _ in range(t):
        c = 0 if c >= 120 else c + 1
    return c


@pytest.mark.parametrize("K", [7, 9])
def test_node_metrics_after_each_chunk_match_reference(K):
    """The verdict's pin: nodeMetricsCur after every 7-segment last=false chunk equals the
    reference's (stream_metrics.npz), renormCounter its phase, and the final last=true call
    the reference's decode."""
    z = load_golden("stream_metrics.npz")
    leg = Legacy(f"k{K}")
    N = 1 << (K - 1)
    for f in range(4):
        rx, met, dec = z[f"k{K}_f{f}_rx"], z[f"k{K}_f{f}_metrics"], z[f"k{K}_f{f}_decoded"]
        reset = leg.metrics_cur()
        assert reset[0] == 0 and (reset[1:] == (N + 1) % 256).all()
        out = np.zeros(dec.shape, np.uint8)
        for c in range(met.shape[0]):
            assert leg.call(rx[7 * c:7 * (c + 1)], out, False) == 0
            assert (leg.metrics_cur() == met[c]).all(), (K, f, c)
            assert leg.renorm_counter() == _renorm_phase(7 * (c + 1))
            assert leg.iteration() == 7 * (c + 1)
        r = leg.call(rx[7 * met.shape[0]:], out, True)
        assert r == dec.shape[0] and (out == dec).all()
        assert leg.iteration() == 0 and leg.renorm_counter() == 0  # reset after last, as :259


@pytest.mark.parametrize("name", sorted(GENK_REF_PARAMS))
def test_genk_node_metrics_and_decode_through_legacy_api(orc, name):
    """k>1 through VITERBI_DECODER_HARD (= viterbiDecoderHard): nodeMetricsCur after every
    chunk equals the reference generic decoder's (genk_metrics.npz); the last=true call
    decodes the staged frame on the GPU, bit-exact against the oracle's ML decode."""
    z = load_golden("genk_metrics.npz")
    leg = Legacy(name)
    k, K, g = GENK_REF_PARAMS[name]
    for f in range(4):
        rx, met, unc = z[f"{name}_f{f}_rx"], z[f"{name}_f{f}_metrics"], z[f"{name}_f{f}_unc"]
        L = 8 * len(unc)
        out = np.zeros(len(unc), np.uint8)
        nfull = (len(rx) - 1) // 7  # chunks before the last call
        for c in range(nfull):
            assert leg.call(rx[7 * c:7 * (c + 1)], out, False) == 0
            assert (leg.metrics_cur() == met[c]).all(), (name, f, c)
        r = leg.call(rx[7 * nfull:], out, True)
        assert r == L // 8
        want = orc.genk_decode(k, K, g, rx[None], L)[0]
        assert (out == want).all(), (name, f)


@pytest.mark.parametrize("name", sorted(GENK_REF_PARAMS))
def test_genk_whole_frames_through_legacy_api(orc, name):
    leg = Legacy(name)
    k, K, g = GENK_REF_PARAMS[name]
    L = 1032 if k == 3 else 1024
    unc, rx = genk_frames(orc, k, K, g, L, 6, 0.03, 77)
    want = orc.genk_decode(k, K, g, rx, L)
    for f in range(rx.shape[0]):
        out = np.zeros(L // 8, np.uint8)
        assert leg.call(rx[f], out, True) == L // 8
        assert (out == want[f]).all()


def _metrics_k1(K, g, seg, m, counter):
    from convolutionalencdec_amd import native

    lib = native.lib()
    c = native.VtbCode.make(K, g)
    cnt = ctypes.c_uint32(counter)
    seg = np.ascontiguousarray(seg, np.uint8)
    m = np.ascontiguousarray(m, np.uint8).copy()
    assert lib.vtb_legacy_metrics_k1(ctypes.byref(c), vp(seg), len(seg), vp(m), ctypes.byref(cnt)) == 0
    return m, cnt.value


@pytest.mark.parametrize("K,g", [(3, (0b111, 0b110)), (3, (0b111, 0b101)), (5, CODES[5]), (7, CODES[7]),
                                 (9, CODES[9])])
def test_metrics_k1_random_chunkings_vs_oracle(orc, K, g):
    """vtb_legacy_metrics_k1 over random chunkings (1..400 segments, renormalisations inside
    chunks) against the oracle's uint8 streaming restatement; (0b111, 0b110) is the
    reference's non-symmetric handTraced code, where the butterfly identity is applied as
    the reference applies it."""
    rng = np.random.default_rng(K)
    L = 2000
    unc, rx = random_frames(orc, K, L, 2, 0.08, K + 3) if g == CODES.get(K) else (None, None)
    if rx is None:
        rx = rng.integers(0, 4, (2, L + K - 1), dtype=np.uint8)
    N = 1 << (K - 1)
    for f in range(rx.shape[0]):
        st = orc.stream(K, g)
        m = np.array([0] + [(N + 1) & 255] * (N - 1), np.uint8)
        counter, pos = 0, 0
        while pos < rx.shape[1] - 1:
            n = int(min(rng.integers(1, 400), rx.shape[1] - 1 - pos))
            seg = rx[f, pos:pos + n]
            m, counter = _metrics_k1(K, g, seg, m, counter)
            _, want = st.decode(seg, np.zeros(4096, np.uint8), False)
            assert (m == want).all(), (K, g, f, pos)
            pos += n
            assert counter == _renorm_phase(pos)


def _reference_program(name, timeout):
    """A reference test program built unchanged against the drop-in (oracle/Makefile
    `harness`: make -C oracle harness, in the build container; the binary travels with the
    tree).  Returns (exit status, stdout)."""
    import subprocess

    from helpers import REPO

    exe = os.path.join(REPO, "oracle", "_ref", name)
    if not os.path.exists(exe):
        pytest.fail(f"{exe} not built (make -C oracle harness where the reference sources are)")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=timeout)
    return r.returncode, r.stdout + r.stderr


def test_reference_handtraced_program_on_gpu():
    """handTracedTest/handTraced.c, unchanged, with its K=3 test code (0b111, 0b110): its
    encoder known answer passes (its own asserts), then viterbiConfigCheck stops it with exit
    status 1, as the reference's own check does for this code (viterbiDecoder.c:15-26 under
    USE_POLY_SYMMETRY, which viterbiDecoder.h:39 defines): the drop-in keeps the reference's
    error behaviour.  The program's decoder known answers are checked below through the
    drop-in's entry points."""
    rc, out = _reference_program("handTraced_amd", 120)
    assert rc == 1, out[-2000:]
    assert "Encoded: 0x68, Got 10 coded segments" in out
    assert "Polynomial 1 does not depend on the input bit and the last bit, therefore polynomial symmetry cannot be used" in out


def test_handtraced_node_metric_known_answers():
    """handTraced.c:70-111's hand-traced node metrics after each of four one-segment
    last=false calls on its corrupted frame: the reference's own known answers, literally,
    through the drop-in's generic-trellis metric update (vtb_legacy_metrics_genk with k = 1,
    the update of viterbiDecoderHard, viterbiDecoder.c:84-131, which handTraced's Makefile
    builds).  The butterfly update (vtb_legacy_metrics_k1, like viterbiDecoderButterflyk1.c)
    assumes generator symmetry this code lacks (the reason viterbiConfigCheck refuses it) and
    differs from the hand trace at state 3 after the first segment (6, not 5); the random
    chunkings test above pins that form to the oracle."""
    from convolutionalencdec_amd import native

    g = (0b111, 0b110)
    code = native.VtbGenKCode.make(1, 3, g)
    corrupted = np.array([0b01, 0b11, 0b01, 0b10, 0b10, 0b11, 0b01, 0, 0, 0], np.uint8)
    m = np.array([0, 5, 5, 5], np.uint32)  # after VITERBI_RESET (handTraced.c:72-75)
    want = [[1, 1, 6, 5], [3, 1, 1, 3], [1, 3, 2, 2], [2, 2, 2, 4]]  # [0], [1], [2], [3]
    for i in range(4):
        seg = np.ascontiguousarray(corrupted[i:i + 1])
        assert native.lib().vtb_legacy_metrics_genk(ctypes.byref(code), vp(seg), 1, vp(m), None) == 0
        assert m.tolist() == want[i], (i, m.tolist())
    k1, _ = _metrics_k1(3, g, corrupted[:1], np.array([0, 5, 5, 5], np.uint8), 0)
    assert k1.tolist() == [1, 1, 6, 6]


def test_reference_bertestk7_program_on_gpu():
    """berTestK7/berTestK7.c, unchanged: 3 x 10,000 2,048-bit frames (glibc rand() channel at
    the three BSC points) decoded one frame per call through the drop-in on the GPU; its own
    pass criterion, and the decoded bit errors equal to the reference's run (92418 / 9655 /
    655)."""
    from helpers import BERTEST_ERRORS

    rc, out = _reference_program("berTestK7_amd", 300)
    assert rc == 0, out[-2000:]
    assert "Success!" in out, out[-2000:]
    rows = [ln.split("|") for ln in out.splitlines() if ln.count("|") == 2 and ln.strip()[:1] in "-0123456789"]
    decoded_errors = tuple(int(r[2].split()[2]) for r in rows)
    assert decoded_errors == BERTEST_ERRORS, (decoded_errors, out[-2000:])


@pytest.mark.parametrize("threads,frames", [(1, 10), (12, 15)])
def test_rand_stream_kept_across_threads(threads, frames):
    """many threads decoding through VITERBI_DECODER_HARD at once keep the
    caller's glibc rand() stream (the draws after the threads continue the stream from before
    them) and leave the process's random state where it was, not in a thread's or the
    library's memory (tests/native/legacy_rand_mt.c, built by `make testprogs`)."""
    import subprocess

    from helpers import REPO

    exe = os.path.join(REPO, "tests", "native", "build", "legacy_rand_mt")
    if not os.path.exists(exe):
        pytest.fail(f"{exe} not built (make testprogs)")
    r = subprocess.run([exe, str(threads), str(frames)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "OK" in r.stdout, (r.stdout + r.stderr)[-2000:]


@pytest.mark.parametrize("name", sorted(GENK_REF_PARAMS))
def test_genk_byte_count_contract(orc, name, capfd):
    """the k>1 drop-in's per-call byte counts ('k > 1: bytes per
    call'): every last=false call returns 0 whatever the chunking, the last=true call returns
    the whole frame's (segments - S) k / 8 bytes equal to the oracle's decode, and a frame whose
    (segments - S) k is not a multiple of 8 prints a message and returns 0, writing nothing."""
    leg = Legacy(name)
    k, K, g = GENK_REF_PARAMS[name]
    L = 1032 if k == 3 else 1024
    unc, rx = genk_frames(orc, k, K, g, L, 2, 0.04, 5)
    want = orc.genk_decode(k, K, g, rx, L)
    rng = np.random.default_rng(k)
    for f in range(rx.shape[0]):
        out = np.zeros(L // 8, np.uint8)
        pos, total = 0, 0
        while pos < rx.shape[1]:
            n = int(min(rng.integers(1, 300), rx.shape[1] - pos))
            last = pos + n == rx.shape[1]
            r = leg.call(rx[f, pos:pos + n], out, last)
            assert r == (L // 8 if last else 0), (name, pos, n, r)
            total += r
            pos += n
        assert total == L // 8 and (out == want[f]).all()
    # a frame one info segment short of whole bytes: message, 0, nothing written
    S = K - 1
    bad = rx[0, : rx.shape[1] - 1]  # (segments - S) k = L - k, not a multiple of 8
    out = np.full(L // 8, 0xA5, np.uint8)
    capfd.readouterr()
    assert leg.call(bad, out, True) == 0
    assert (out == 0xA5).all()
    assert "does not hold a whole number of bytes" in capfd.readouterr().out
    assert leg.iteration() == 0  # reset after last
    assert (len(bad) - S) * k % 8 != 0
