"""GPU: the general rate-k/n decoder (vtb_genk_decode_device) against the
checker's oracle_genk_decode on noisy frames, bit for bit; k = 1 against the k=1 batch
decoder (pinned by the reference's golden vectors); strided rows."""
import ctypes

import numpy as np
import pytest

from helpers import CODES, GENK_CODES, Oracle, genk_frames, golden_sets

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from convolutionalencdec_amd import ConvCode, GenKDecoder, ViterbiDecoder, native  # noqa: E402


@pytest.fixture(scope="module")
def orc():
    return Oracle()


@pytest.fixture(scope="module", autouse=True)
def gpu_present():
    if not torch.cuda.is_available() or native.lib().vtb_device_count() < 1:
        pytest.fail("no gfx950 GPU visible to the C ABI (GPU tests must not silently pass)")


@pytest.mark.parametrize("code", GENK_CODES, ids=lambda c: f"k{c[0]}K{c[1]}n{len(c[2])}")
@pytest.mark.parametrize("L,F,p", [(48, 7, 0.1), (1032, 300, 0.04), (2040, 65, 0.0), (16320, 5, 0.04), (16368, 3, 0.0)])
def test_genk_gpu_vs_oracle(orc, code, L, F, p):
    k, K, g = code
    unc, coded = genk_frames(orc, k, K, g, L, F, p, L + F + k)
    want = orc.genk_decode(k, K, g, coded, L)
    d = GenKDecoder(k, K, g, L)
    got = d.decode_device(torch.from_numpy(coded).cuda()).cpu().numpy()
    bad = np.flatnonzero((got != want).any(axis=1))
    assert bad.size == 0, (code, L, bad.size, bad[:8])
    if p == 0.0:
        assert (got == unc).all()  # noise-free frames decode to their payload


@pytest.mark.parametrize("code", GENK_CODES, ids=lambda c: f"k{c[0]}K{c[1]}n{len(c[2])}")
def test_genk_gpu_window_phases(orc, code):
    """Frame lengths of every residue T mod S (the first survivor-pointer window is partial,
    or the boundaries fall on other steps) and of one and two segments."""
    k, K, g = code
    S = K - 1
    for m in sorted({1, 2, 3, 5, 7, 11, 13, 2 * S + 1, 3 * S + 2, 64, 255}):
        L = k * m
        # received segments at random (any sequence is a valid decoder input; the encoder
        # helpers work in whole payload bytes)
        rng = np.random.default_rng(1000 + m)
        coded = rng.integers(0, 1 << len(g), (9, m + S), dtype=np.uint8)
        want = orc.genk_decode(k, K, g, coded, L)
        xi = torch.from_numpy(coded).cuda()
        out = torch.zeros((coded.shape[0], (L + 7) // 8), dtype=torch.uint8, device="cuda")
        gk = native.VtbGenKCode.make(k, K, g)  # the C ABI: any multiple of k (GenKDecoder keeps 8 | L)
        native.check(native.lib().vtb_genk_decode_device(ctypes.byref(gk), L, ctypes.c_void_p(xi.data_ptr()),
                                                         xi.stride(0), ctypes.c_void_p(out.data_ptr()),
                                                         out.stride(0), coded.shape[0], None), "vtb_genk_decode_device")
        got = out.cpu().numpy()
        bad = np.flatnonzero((got != want).any(axis=1))
        assert bad.size == 0, (code, L, bad[:8])


def test_genk_gpu_k1_golden_vectors():
    """k = 1, K = 7: the reference's own golden frames decode to the reference's output."""
    for key, L, unc, rx, dec in golden_sets(7):
        if L % 8:
            continue
        d = GenKDecoder(1, 7, CODES[7], L)
        got = d.decode_device(torch.from_numpy(np.ascontiguousarray(rx)).cuda()).cpu().numpy()
        assert (got == dec).all(), key


def test_genk_gpu_k1_equals_batch_decoder(orc):
    from helpers import random_frames

    L = 1024
    unc, x = random_frames(orc, 7, L, 200, 0.06, 99)
    xt = torch.from_numpy(np.ascontiguousarray(x)).cuda()
    a = GenKDecoder(1, 7, CODES[7], L).decode_device(xt).cpu().numpy()
    b = ViterbiDecoder(ConvCode(7, CODES[7]), frame_bits=L).decode_device(xt).cpu().numpy()
    assert (a == b).all()


def test_genk_gpu_strided_rows(orc):
    k, K, g = GENK_CODES[0]
    L, F = 512, 33
    unc, coded = genk_frames(orc, k, K, g, L, F, 0.05, 4)
    T = coded.shape[1]
    xi = torch.zeros((F, T + 29), dtype=torch.uint8, device="cuda")
    xi[:, :T] = torch.from_numpy(coded).cuda()
    out = torch.full((F, L // 8 + 7), 0xA5, dtype=torch.uint8, device="cuda")
    code = native.VtbGenKCode.make(k, K, g)
    native.check(native.lib().vtb_genk_decode_device(ctypes.byref(code), L, ctypes.c_void_p(xi.data_ptr()), xi.stride(0),
                                                     ctypes.c_void_p(out.data_ptr()), out.stride(0), F, None),
                 "vtb_genk_decode_device")
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    assert (got[:, L // 8:] == 0xA5).all()
    assert (got[:, :L // 8] == orc.genk_decode(k, K, g, coded, L)).all()


def _random_codes(seed, count):
    """Random (k, K, generators) inside the C ABI's limits (k (K-1) <= 8, k K <= 12, n <= 8):
    every ACS path of the kernel -- N <= 64 and N = 256, packed (n <= 3) and linear labels."""
    rng = np.random.default_rng(seed)
    out = []
    while len(out) < count:
        k = int(rng.integers(1, 5))
        K = int(rng.integers(2, 8 // k + 2))
        if k * (K - 1) > 8 or k * K > 12:
            continue
        n = int(rng.integers(1, 9))
        g = tuple(int(v) for v in rng.integers(1, 1 << (k * K), n))
        out.append((k, K, g))
    return out


@pytest.mark.parametrize("code", _random_codes(20261017, 40), ids=lambda c: f"k{c[0]}K{c[1]}n{len(c[2])}")
def test_genk_gpu_random_codes(orc, code):
    """Random codes (any generator set, n = 1..8, incl. catastrophic and repeated generators),
    random received segments and encoded noisy frames, several lengths: bit for bit against
    oracle_genk_decode."""
    k, K, g = code
    S, n = K - 1, len(g)
    rng = np.random.default_rng(sum(g) + 31 * k + K)
    for m in (1, 7, 64, 517):
        L = k * m
        coded = rng.integers(0, 1 << n, (6, m + S), dtype=np.uint8)
        if L % 8 == 0:  # encoded frames with light noise (decisions not all ties)
            _, enc = genk_frames(orc, k, K, g, L, 3, 0.03, m)
            coded = np.concatenate([coded, enc])
        want = orc.genk_decode(k, K, g, coded, L)
        xi = torch.from_numpy(coded).cuda()
        out = torch.zeros((coded.shape[0], (L + 7) // 8), dtype=torch.uint8, device="cuda")
        gk = native.VtbGenKCode.make(k, K, g)
        native.check(native.lib().vtb_genk_decode_device(ctypes.byref(gk), L, ctypes.c_void_p(xi.data_ptr()),
                                                         xi.stride(0), ctypes.c_void_p(out.data_ptr()),
                                                         out.stride(0), coded.shape[0], None), "vtb_genk_decode_device")
        got = out.cpu().numpy()
        bad = np.flatnonzero((got != want).any(axis=1))
        assert bad.size == 0, (code, L, bad[:8])


@pytest.mark.parametrize("seed", range(6))
def test_genk_gpu_random_k1_reference_u8(orc, seed):
    """k = 1 in the reference's uint8 butterfly arithmetic (VTB_GENK_K1_REFERENCE_U8) for
    random codes of K = 3..9, n = 1..8 (sums that wrap mod 256 for n >= 4), against
    oracle_k1n_decode."""
    rng = np.random.default_rng(700 + seed)
    for _ in range(4):
        K = int(rng.integers(3, 10))
        n = int(rng.integers(1, 9))
        g = tuple(int(v) for v in rng.integers(1, 1 << K, n))
        L = int(rng.integers(1, 700))
        coded = rng.integers(0, 256, (5, L + K - 1), dtype=np.uint8)  # garbage high bits too
        want = orc.k1n_decode(K, g, coded, L)
        code = native.VtbGenKCode.make(1, K, g, native.VTB_GENK_K1_REFERENCE_U8)
        xi = torch.from_numpy(coded).cuda()
        out = torch.zeros((coded.shape[0], (L + 7) // 8), dtype=torch.uint8, device="cuda")
        native.check(native.lib().vtb_genk_decode_device(ctypes.byref(code), L, ctypes.c_void_p(xi.data_ptr()),
                                                         xi.stride(0), ctypes.c_void_p(out.data_ptr()),
                                                         out.stride(0), coded.shape[0], None), "vtb_genk_decode_device")
        got = out.cpu().numpy()
        assert (got == want).all(), (K, g, L)
