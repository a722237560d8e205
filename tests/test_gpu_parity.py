"""GPU parity: the HIP decoder (called through the C ABI) against the reference's golden
vectors, the reference's berTestK7 known-answer counts and the oracle on seeded inputs.
Bit-exact everywhere (integer work)."""
import ctypes
import os

import numpy as np
import pytest

from helpers import (BERTEST_ERRORS, CODES, Oracle, golden_sets, hard_to_soft, load_golden, manifest, random_frames)

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from convolutionalencdec_amd import ConvCode, ViterbiDecoder, decode_multi, native  # noqa: E402

# "auto": the library's own choice; the others force one kernel family: "k7" (K=7,
# survivors in LDS), "gws" (the same K=7 kernel with survivors in a global workspace), "k9"
# (K=9, survivors in a global workspace), "lds" (every K).
# "k7s": the K=7 persistent split kernel (one frame per wave as two halves, unconverged frames
# re-decoded from a list by the global variant) wherever it applies.
# "k9p": the K=9 pair kernel (two frames per wave) also for the batches "k9" / "auto" decode one
# frame per wave (k9s; VTB_DEBUG bit 18).
KERNELS = ("auto", "k7", "gws", "k7s", "k9", "k9p", "lds")


class Kern(str):
    def need(self, K):
        assert K in KS_OF.get(str(self), (K,)), (self, K)  # (combinations are generated valid)

    def ran(self):
        """The last decode ran the forced family (plans capture VTB_KERNEL at creation: a stale
        plan would otherwise pass on another kernel)."""
        want = FAMILY_INSTANCES.get(str(self))
        if want:
            assert native.last_kernel() in want, (str(self), native.last_kernel())


KS_OF = {"k7": (7,), "gws": (7,), "k7s": (7,), "k9": (9,), "k9p": (9,)}  # kernel families tied to one K
# the kernel instances (vtb_debug_last_kernel) each forced family may run
FAMILY_INSTANCES = {"k7": ("k7_lds", "k7_lds_loop", "k7_lds_split"), "gws": ("k7_global", "k7_global_loop"),
                    "k9": ("k9", "k9_loop", "k9s"), "k9p": ("k9", "k9_loop"), "lds": ("lds_path", "lds_path_gs")}


K9_PAIR = 1 << 18


def kernels_for(K):
    return [k for k in KERNELS if K in KS_OF.get(k, (K,))]


def kk(Ks):
    """(K, kernel) pairs: every kernel family that decodes K."""
    return [(K, k) for K in Ks for k in kernels_for(K)]


@pytest.fixture(scope="module")
def orc():
    return Oracle()


@pytest.fixture(scope="module", autouse=True)
def gpu_present():
    if not torch.cuda.is_available() or native.lib().vtb_device_count() < 1:
        pytest.fail("no gfx950 GPU visible to the C ABI (GPU tests must not silently pass)")


@pytest.fixture
def kernel(request, monkeypatch):
    if request.param == "auto":
        monkeypatch.delenv("VTB_KERNEL", raising=False)
    elif request.param == "k9p":
        monkeypatch.setenv("VTB_KERNEL", "k9")
        monkeypatch.setenv("VTB_DEBUG", str(K9_PAIR))
    else:
        monkeypatch.setenv("VTB_KERNEL", request.param)
    return Kern(request.param)


def dev_decode(dec, frames):
    x = torch.from_numpy(np.ascontiguousarray(frames).reshape(frames.shape[0], -1)).cuda()
    out = dec.decode_device(x)
    torch.cuda.synchronize()
    return out.cpu().numpy()


@pytest.mark.parametrize("K,kernel", kk([5, 7, 9]), indirect=["kernel"])
def test_hard_golden_vectors(K, kernel):
    kernel.need(K)
    for key, L, unc, rx, dec in golden_sets(K):
        d = ViterbiDecoder(ConvCode(K, CODES[K]), frame_bits=L)
        assert (d.decode_host(rx) == dec).all(), (K, key)
        assert (dev_decode(d, rx) == dec).all(), (K, key)
        kernel.ran()


@pytest.mark.parametrize("K,kernel", kk([5, 7, 9]), indirect=["kernel"])
def test_soft_bridge_golden_vectors(K, kernel):
    """Soft input q = 255*bit must reproduce the reference's hard decode bit for bit."""
    kernel.need(K)
    for key, L, unc, rx, dec in golden_sets(K):
        d = ViterbiDecoder(ConvCode(K, CODES[K]), frame_bits=L, soft=True)
        assert (dev_decode(d, hard_to_soft(rx)) == dec).all(), (K, key)


@pytest.mark.parametrize("K,g,kernel", [(K, g, k) for K, g in [(3, (0b111, 0b101)), (4, (0o15, 0o17)), (5, CODES[5]),
                                                              (6, (0o53, 0o75)), (7, CODES[7]), (8, (0o247, 0o371)),
                                                              (9, CODES[9])] for k in kernels_for(K)],
                         indirect=["kernel"])
@pytest.mark.parametrize("L", [1, 7, 100, 1001, 2048, 4096, 9000, 16383, 16384])
def test_hard_random_vs_oracle(orc, K, g, L, kernel):
    """Every k = 1 rate-1/2 constraint length at every frame length up to VTB_MAX_FRAME_BITS
    (the reference's MAX_PKT_LEN_UNCODED_BITS, viterbiDecoder.h:18) on every kernel family that
    decodes it; the generic kernel's GS variant takes the frames its LDS variant cannot hold."""
    kernel.need(K)
    if kernel == "k7" and L > 9000:
        # the forced K=7 LDS-resident kernel holds frames up to its LDS capacity:
        # refused with an error code, never a wrong result (the library's own choice takes them)
        unc, rx = random_frames(orc, K, L, 3, 0.06, 12 + L, g=g)
        with pytest.raises(native.VtbError) as e:
            ViterbiDecoder(ConvCode(K, g), frame_bits=L).decode_host(rx)
        assert e.value.code == native.VTB_ERR_UNSUPPORTED
        return
    for p, seed in ((0.0, 11), (0.06, 12), (0.5, 13)):
        unc, rx = random_frames(orc, K, L, 257, p, seed + L, g=g)
        expect = orc.decode(K, g, rx, L)
        got = ViterbiDecoder(ConvCode(K, g), frame_bits=L).decode_host(rx)
        assert (got == expect).all(), (K, L, p)
        kernel.ran()
        if p == 0.0:
            assert (got == unc).all()


@pytest.mark.parametrize("K,kernel", kk([5, 7, 9]), indirect=["kernel"])
@pytest.mark.parametrize("L", [9, 1024, 2048])
def test_soft_random_vs_oracle(orc, K, L, kernel):
    kernel.need(K)
    for sigma, seed in ((0.4994, 21), (0.6287, 22), (1.5, 23)):
        unc, q = random_frames(orc, K, L, 193, 0.0, seed + L, soft=True, sigma=sigma)
        expect = orc.decode(K, CODES[K], q, L, soft=True)
        got = dev_decode(ViterbiDecoder(ConvCode(K, CODES[K]), frame_bits=L, soft=True), q)
        assert (got == expect).all(), (K, L, sigma)
        kernel.ran()


@pytest.mark.parametrize("soft", [False, True])
@pytest.mark.parametrize("L", [234, 235, 500, 1051, 1519, 2203, 2970])
def test_split_frames_vs_oracle(orc, L, soft):
    """Small K=7 batches decode each frame in one wave as two halves at once (DESIGN.md 4.1,
    split frames): the frame-length limits of that mode (T = 240, t1 = 1536), clean, noisy and
    pure-noise frames (the halves' metrics then rarely converge: the unsplit re-decode), an
    odd count, and one frame alone -- against the oracle.  L = 1051 and 2203 (T = 1 mod 96):
    T + 96 odd with (T + 95) / 2 a multiple of 48, where a floored t1 left the second half one
    step short of the frame's end (found by the round-2 fuzz sweep, seed 31337 case 1947)."""
    K = 7
    code = ConvCode(K, CODES[K])
    d = ViterbiDecoder(code, frame_bits=L, soft=soft)
    for noise, seed in ((0.0, 1), (0.05, 2), (0.5, 3)):
        if soft:
            unc, x = random_frames(orc, K, L, 65, 0.0, 50 + seed + L, soft=True, sigma=(0.3, 0.63, 4.0)[seed - 1])
        else:
            unc, x = random_frames(orc, K, L, 65, noise, 50 + seed + L)
        want = orc.decode(K, CODES[K], x, L, soft=soft)
        assert (dev_decode(d, x) == want).all(), (L, soft, seed)
        assert (dev_decode(d, x[:1]) == want[:1]).all(), (L, soft, seed)


@pytest.mark.parametrize("soft", [False, True])
@pytest.mark.parametrize("L", [1915, 2059])
@pytest.mark.parametrize("kernel", ["auto", "k7s"], indirect=True)
def test_split_loop_odd_tail(orc, L, soft, kernel):
    """The persistent split kernel at frame lengths where a floored t1 left
    the second half one step short of T - 1: L = 1915 (T = 1 mod 96, warm-up 96; the kernel
    decodes it) and L = 2059 (T = 49 mod 96, warm-up 48: with the correct t1 its halves no
    longer fit 8 waves per CU, so the global-survivor variant decodes it).  Soft input takes
    the split kernel by default, hard input under k7s."""
    K, F = 7, 4096
    if soft:
        unc, x = random_frames(orc, K, L, F, 0.0, 880 + L, soft=True, sigma=0.55)
    else:
        unc, x = random_frames(orc, K, L, F, 0.03, 880 + L)
    want = orc.decode(K, CODES[K], x, L, soft=soft, threads=16)
    got = dev_decode(ViterbiDecoder(ConvCode(K, CODES[K]), frame_bits=L, soft=soft), x)
    bad = np.flatnonzero((got != want).any(axis=1))
    assert bad.size == 0, (L, soft, bad.size, bad[:8])


@pytest.mark.parametrize("soft", [False, True])
@pytest.mark.parametrize("K,L,F,kernel", [(K, L, F, k) for K, L, F in [(7, 1024, 12289), (7, 1024, 40961), (9, 512, 20481)]
                                          for k in kernels_for(K) if k != "lds" and not (k == "k7" and F > 20000)],
                         indirect=["kernel"])
def test_persistent_grid_many_pairs_per_wave(orc, K, L, F, soft, kernel):
    """Batches with several frame pairs per wave of the persistent grid (more pairs than the
    CUs hold at once), an odd frame count (the last pair has one frame), the next pair's
    input prefetched during a traceback: the whole batch against the oracle."""
    from convolutionalencdec_amd import frames as devframes

    kernel.need(K)
    code = ConvCode(K, CODES[K])
    unc, rx = devframes.make_frames(code, F, L, soft=soft, snr_db=-4.0, p=0.04, seed=F + K)
    d = ViterbiDecoder(code, frame_bits=L, soft=soft)
    got = d.decode_device(rx.reshape(F, -1)).cpu().numpy()
    ref = orc.decode(K, CODES[K], rx.reshape(F, -1).cpu().numpy(), L, soft=soft, threads=min(16, os.cpu_count() or 1))
    bad = np.flatnonzero((got != ref).any(axis=1))
    assert bad.size == 0, (bad.size, bad[:8])


@pytest.mark.parametrize("soft", [False, True])
@pytest.mark.parametrize("L", [10000, 16384])
@pytest.mark.parametrize("kernel", [k for k in kernels_for(7) if k != "k7"], indirect=True)
def test_k7_long_frames_vs_oracle(orc, L, soft, kernel):
    """Frames past the LDS-resident kernel's survivor capacity up to the API maximum
    (VTB_MAX_FRAME_BITS, reference viterbiDecoder.h:18): the global-survivor variant."""
    K = 7
    kernel.need(K)
    if soft:
        unc, x = random_frames(orc, K, L, 67, 0.0, 31 + L, soft=True, sigma=0.6287)
    else:
        unc, x = random_frames(orc, K, L, 67, 0.05, 31 + L)
    d = ViterbiDecoder(ConvCode(K, CODES[K]), frame_bits=L, soft=soft)
    assert (dev_decode(d, x) == orc.decode(K, CODES[K], x, L, soft=soft)).all()


@pytest.mark.parametrize("soft", [False, True])
@pytest.mark.parametrize("L", [4095, 16384])
@pytest.mark.parametrize("kernel", kernels_for(9), indirect=True)
def test_k9_long_frames_vs_oracle(orc, L, soft, kernel):
    """K=9 frames up to the API maximum (reference viterbiDecoder.h:18), odd and even T."""
    K = 9
    kernel.need(K)
    if soft:
        unc, x = random_frames(orc, K, L, 33, 0.0, 41 + L, soft=True, sigma=0.6287)
    else:
        unc, x = random_frames(orc, K, L, 33, 0.04, 41 + L)
    d = ViterbiDecoder(ConvCode(K, CODES[K]), frame_bits=L, soft=soft)
    assert (dev_decode(d, x) == orc.decode(K, CODES[K], x, L, soft=soft)).all()


@pytest.mark.parametrize("K,kernel", kk([7, 9]), indirect=["kernel"])
def test_soft_extreme_values(orc, K, kernel):
    """Saturated, constant and alternating soft inputs (tie-heavy) match the oracle."""
    kernel.need(K)
    L = 512
    T = L + K - 1
    rng = np.random.default_rng(7)
    cases = [np.zeros((4, T, 2), np.uint8), np.full((4, T, 2), 255, np.uint8), np.full((4, T, 2), 128, np.uint8),
             np.full((4, T, 2), 127, np.uint8), rng.choice(np.array([0, 127, 128, 255], np.uint8), (64, T, 2))]
    d = ViterbiDecoder(ConvCode(K, CODES[K]), frame_bits=L, soft=True)
    for q in cases:
        assert (dev_decode(d, q) == orc.decode(K, CODES[K], q, L, soft=True)).all()


@pytest.mark.parametrize("kernel", kernels_for(7), indirect=True)
def test_bertest_k7_kat_on_gpu(orc, kernel):
    """The reference berTestK7 stream (glibc rand seed 9865, 3 x 10000 packets) decoded on
    the GPU gives exactly the reference's decoded bit-error counts."""
    kernel.need(7)
    unc, rx, _ = orc.bertest()
    d = ViterbiDecoder(ConvCode(7, CODES[7]), frame_bits=2048)
    for c in range(3):
        out = dev_decode(d, rx[c])
        assert int(np.unpackbits(unc[c] ^ out).sum()) == BERTEST_ERRORS[c]


def test_full_size_soft_batch_properties(orc):
    """BASELINE config C3 at full size: 65536 x 2048-bit soft frames.  Noise-free frames
    decode to the payload exactly; a noisy batch decodes identically on two launches and a
    strided subset matches the oracle."""
    from helpers import encode_bits

    K, L, F, U = 7, 2048, 65536, 4096
    rng = np.random.default_rng(2024)
    unc = rng.integers(0, 256, (U, L // 8), dtype=np.uint8)
    q = hard_to_soft(encode_bits(K, CODES[K], np.unpackbits(unc, axis=1)))
    d = ViterbiDecoder(ConvCode(K, CODES[K]), frame_bits=L, soft=True)
    x = torch.from_numpy(q.reshape(U, -1)).cuda().repeat(F // U, 1)
    out = d.decode_device(x).cpu().numpy()
    assert (out == np.tile(unc, (F // U, 1))).all()
    noisy = np.clip(q.astype(np.int16) + rng.integers(-150, 150, q.shape, dtype=np.int16), 0, 255).astype(np.uint8)
    xn = torch.from_numpy(noisy.reshape(U, -1)).cuda().repeat(F // U, 1)
    o1 = d.decode_device(xn)
    o2 = d.decode_device(xn)
    torch.cuda.synchronize()
    assert torch.equal(o1, o2)
    o1 = o1.cpu().numpy()
    assert (o1[:U] == o1[F - U:]).all()
    sub = np.arange(0, U, 61)
    assert (o1[sub] == orc.decode(K, CODES[K], noisy[sub], L, soft=True)).all()


@pytest.mark.parametrize("soft", [False, True])
@pytest.mark.parametrize("kernel", kernels_for(9), indirect=True)
def test_k9_full_config(orc, kernel, soft):
    """C4: K=9, 4096 x 1024 -- every frame against the oracle (hard at BSC p = 0.03, soft at
    the bench's SNR), and the decoded BER."""
    K, L, F = 9, 1024, 4096
    kernel.need(K)
    if soft:
        unc, rx = random_frames(orc, K, L, F, 0.0, 99, soft=True, sigma=0.63)
    else:
        unc, rx = random_frames(orc, K, L, F, 0.03, 99)
    got = ViterbiDecoder(ConvCode(K, CODES[K]), frame_bits=L, soft=soft).decode_host(rx)
    ref = orc.decode(K, CODES[K], rx, L, soft=soft, threads=16)
    mism = np.flatnonzero((got != ref).any(axis=1))
    assert mism.size == 0, f"{mism.size} of {F} frames differ (first {mism[:8]})"
    ber = np.unpackbits(got ^ unc).mean()
    assert ber < 1e-3


@pytest.mark.parametrize("soft", [False, True])
def test_host_path_chunked(orc, soft):
    """vtb_decode_host on a batch large enough to run in overlapped chunks (H2D of one chunk
    beside the decode of the previous, a partial last chunk): identical to the device path
    and to the oracle."""
    K, L, F = 7, 256, 40961
    rng = np.random.default_rng(5 + soft)
    T = L + K - 1
    x = rng.integers(0, 256, (F, 2 * T if soft else T), dtype=np.uint8)
    if not soft:
        x &= 3
    d = ViterbiDecoder(ConvCode(K, CODES[K]), frame_bits=L, soft=soft)
    host = d.decode_host(x)
    assert (host == dev_decode(d, x)).all()
    sub = np.r_[0:64, F - 64:F]
    assert (host[sub] == orc.decode(K, CODES[K], x[sub], L, soft=soft)).all()


def test_strided_device_io(orc):
    K, L, F = 7, 640, 300
    unc, rx = random_frames(orc, K, L, F, 0.05, 5)
    T = L + K - 1
    big = np.zeros((F, T + 37), np.uint8)
    big[:, :T] = rx
    d = ViterbiDecoder(ConvCode(K, CODES[K]), frame_bits=L)
    x = torch.from_numpy(big).cuda()[:, :T]
    out = torch.zeros((F, 128), dtype=torch.uint8, device="cuda")
    lib = native.lib()
    rc = lib.vtb_decode_device(d._plan, ctypes.c_void_p(x.data_ptr()), x.stride(0), ctypes.c_void_p(out.data_ptr()),
                               out.stride(0), F, None)
    assert rc == 0
    torch.cuda.synchronize()
    assert (out.cpu().numpy()[:, :L // 8] == orc.decode(K, CODES[K], rx, L)).all()
    assert (out.cpu().numpy()[:, L // 8:] == 0).all()
    # strides smaller than a frame are rejected, zero frames is a no-op
    assert lib.vtb_decode_device(d._plan, ctypes.c_void_p(x.data_ptr()), T - 1, ctypes.c_void_p(out.data_ptr()), 128,
                                 F, None) == native.VTB_ERR_INVALID
    assert lib.vtb_decode_device(d._plan, None, 0, None, 0, 0, None) == 0


def test_multi_device_host_api(orc):
    """vtb_decode_host_multi: first call (plans created), repeated calls on the kept plans with
    larger and smaller batches and another code, and after vtb_release_cached_plans."""
    from convolutionalencdec_amd import release_cached_plans

    K, L, F = 7, 256, 1000
    unc, rx = random_frames(orc, K, L, F, 0.04, 8)
    ref = orc.decode(K, CODES[K], rx, L)
    assert (decode_multi(rx, ConvCode(K, CODES[K]), L) == ref).all()
    assert (decode_multi(rx[:333], ConvCode(K, CODES[K]), L) == ref[:333]).all()
    big = np.concatenate([rx] * 5)
    assert (decode_multi(big, ConvCode(K, CODES[K]), L) == np.concatenate([ref] * 5)).all()
    u9, rx9 = random_frames(orc, 9, L, 300, 0.03, 9)
    assert (decode_multi(rx9, ConvCode(9, CODES[9]), L) == orc.decode(9, CODES[9], rx9, L)).all()
    release_cached_plans()
    assert (decode_multi(rx, ConvCode(K, CODES[K]), L) == ref).all()
    release_cached_plans()


# ---------------- legacy C API (include/viterbiDecoder.h) on the GPU ----------------

def _legacy(K):
    from convolutionalencdec_amd import LIB_DIR

    L = ctypes.CDLL(os.path.join(LIB_DIR, f"libviterbi_legacy_k{K}.so"))
    v = ctypes.c_void_p
    L.viterbiInitButterflyk1.argtypes = [v]
    L.resetViterbiDecoderHardButterflyk1.argtypes = [v]
    L.viterbiDecoderHardButterflyk1.argtypes = [v, v, v, ctypes.c_int, ctypes.c_bool]
    L.viterbiConfigCheck.argtypes = []
    return L


def _state(K):
    size = manifest()["kat"]["viterbiHardState_t_sizeof"][str(K)]
    buf = np.zeros(size + 64, np.uint8)
    off = (-buf.ctypes.data) % 64
    return buf, ctypes.c_void_p(buf.ctypes.data + off)


@pytest.mark.parametrize("K", [5, 7, 9])
def test_legacy_api_golden(K):
    lib = _legacy(K)
    buf, st = _state(K)
    lib.resetViterbiDecoderHardButterflyk1(st)
    lib.viterbiInitButterflyk1(st)
    assert lib.viterbiConfigCheck() == 0
    for key, L, unc, rx, dec in golden_sets(K):
        for f in range(0, rx.shape[0], 5):
            out = np.zeros(dec.shape[1], np.uint8)
            row = np.ascontiguousarray(rx[f])
            r = lib.viterbiDecoderHardButterflyk1(st, row.ctypes.data_as(ctypes.c_void_p),
                                                  out.ctypes.data_as(ctypes.c_void_p), len(row), True)
            assert r == (L - 1) // 8 + 1
            assert (out == dec[f]).all(), (key, f)


def test_legacy_api_streaming_chunks():
    """last=false chunks are accumulated; the last=true call decodes the whole frame."""
    lib = _legacy(7)
    buf, st = _state(7)
    lib.resetViterbiDecoderHardButterflyk1(st)
    lib.viterbiInitButterflyk1(st)
    z = load_golden("stream_metrics.npz")
    rx, dec = z["k7_f0_rx"], z["k7_f0_decoded"]
    out = np.zeros(dec.shape, np.uint8)
    c = 0
    while len(rx) - c > 7:
        chunk = np.ascontiguousarray(rx[c:c + 7])
        assert lib.viterbiDecoderHardButterflyk1(st, chunk.ctypes.data_as(ctypes.c_void_p),
                                                 out.ctypes.data_as(ctypes.c_void_p), 7, False) == 0
        c += 7
    rest = np.ascontiguousarray(rx[c:])
    r = lib.viterbiDecoderHardButterflyk1(st, rest.ctypes.data_as(ctypes.c_void_p), out.ctypes.data_as(ctypes.c_void_p),
                                          len(rest), True)
    assert r == dec.shape[0]
    assert (out == dec).all()
