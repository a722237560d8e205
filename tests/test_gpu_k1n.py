"""k = 1 codes with n != 2 on the GPU.

* The legacy drop-in built for params/k7n3, k9n3, k5n4 and k8n3 (libviterbi_legacy_<name>.so)
  decodes the reference's golden frames (tests/golden/k1n.npz, produced by the reference
  compiled with the same params) through VITERBI_DECODER_HARD exactly, with the reference's
  byte count, and nodeMetricsCur after every 7-segment last=false chunk equals the
  reference's (viterbiDecoderButterflyk1.c:101-191 with its compile-time n).
* vtb_genk_decode_device with VTB_GENK_K1_REFERENCE_U8 equals the oracle's restatement
  (oracle_k1n_decode) on random frames of any length, garbage high bits included; without
  the flag (exact metrics) it equals oracle_genk_decode at any length.
"""
import ctypes

import numpy as np
import pytest

from helpers import K1N_PARAMS, Oracle, k1n_frames, load_golden, vp

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from convolutionalencdec_amd import native  # noqa: E402
from test_gpu_legacy import Legacy  # noqa: E402


@pytest.fixture(scope="module")
def orc():
    return Oracle()


@pytest.fixture(scope="module", autouse=True)
def gpu_present():
    if not torch.cuda.is_available() or native.lib().vtb_device_count() < 1:
        pytest.fail("no gfx950 GPU visible to the C ABI (GPU tests must not silently pass)")


@pytest.mark.parametrize("name", sorted(K1N_PARAMS))
def test_legacy_dropin_decodes_reference_golden(name):
    z = load_golden("k1n.npz")
    leg = Legacy(name)
    keys = sorted({k.rsplit("_", 1)[0] for k in z if k.startswith(name + "_L")})
    assert keys
    for key in keys:
        L = int(key.split("_")[1][1:])
        rx, dec = z[key + "_rx"], z[key + "_decoded"]
        for f in range(rx.shape[0]):
            out = np.zeros(L // 8, np.uint8)
            assert leg.call(rx[f], out, True) == (L - 1) // 8 + 1
            assert (out == dec[f]).all(), (name, key, f)


@pytest.mark.parametrize("name", sorted(K1N_PARAMS))
def test_legacy_node_metrics_after_each_chunk(name):
    z = load_golden("k1n.npz")
    leg = Legacy(name)
    K, g = K1N_PARAMS[name]
    N = 1 << (K - 1)
    for f in range(4):
        rx, met, dec = z[f"{name}_stream_f{f}_rx"], z[f"{name}_stream_f{f}_metrics"], z[f"{name}_stream_f{f}_decoded"]
        reset = leg.metrics_cur()
        assert reset[0] == 0 and (reset[1:] == (N + 1) % 256).all()
        out = np.zeros(dec.shape, np.uint8)
        for c in range(met.shape[0]):
            assert leg.call(rx[7 * c:7 * (c + 1)], out, False) == 0
            assert (leg.metrics_cur() == met[c]).all(), (name, f, c)
        assert leg.call(rx[7 * met.shape[0]:], out, True) == dec.shape[0]
        assert (out == dec).all(), (name, f)


def genk_device(K, g, rx, L, flags):
    code = native.VtbGenKCode.make(1, K, g, flags)
    x = torch.from_numpy(np.ascontiguousarray(rx)).cuda()
    ob = (L + 7) // 8
    out = torch.zeros((rx.shape[0], ob), dtype=torch.uint8, device="cuda")
    rc = native.lib().vtb_genk_decode_device(ctypes.byref(code), L, ctypes.c_void_p(x.data_ptr()), x.stride(0),
                                             ctypes.c_void_p(out.data_ptr()), ob, rx.shape[0], None)
    assert rc == 0, native.strerror(rc)
    torch.cuda.synchronize()
    return out.cpu().numpy()


@pytest.mark.parametrize("name", sorted(K1N_PARAMS))
@pytest.mark.parametrize("L", [1, 13, 64, 1001, 2048])
def test_reference_u8_mode_vs_oracle(orc, name, L):
    K, g = K1N_PARAMS[name]
    for p, seed in ((0.0, 1), (0.06, 2), (0.5, 3)):
        if L % 8 == 0:
            unc, rx = k1n_frames(orc, K, g, L, 24, p, seed + L, garbage=(p == 0.06))
        else:  # odd L: random segment bytes (any input decodes; parity is what counts)
            unc, rx = None, np.random.default_rng(seed + 7 * L).integers(0, 256, (24, L + K - 1), dtype=np.uint8)
        want = orc.k1n_decode(K, g, rx, L)
        got = genk_device(K, g, rx, L, native.VTB_GENK_K1_REFERENCE_U8)
        assert (got == want).all(), (name, L, p)
        exact = genk_device(K, g, rx, L, 0)
        assert (exact == orc.genk_decode(1, K, g, rx, L)).all(), (name, L, p)
        if p == 0.0 and L % 8 == 0:
            assert (got == unc).all()


# ---- K=7 / K=9 rate 1/3 on the K=7 LDS pair kernel / the K=9 frame kernel (NB = 3) ----

N3 = {7: (K1N_PARAMS["k7n3"][1], "k7_lds_n3"), 9: (K1N_PARAMS["k9n3"][1], "k9_n3")}


def genk_device_kernel(K, g, rx, L, flags, monkeypatch=None, force_genk=False):
    """genk_device, also returning the kernel instance the call launched."""
    if force_genk:
        monkeypatch.setenv("VTB_KERNEL", "genk")
    try:
        out = genk_device(K, g, rx, L, flags)
        return out, native.last_kernel()
    finally:
        if force_genk:
            monkeypatch.delenv("VTB_KERNEL")


@pytest.mark.parametrize("K", [7, 9])
@pytest.mark.parametrize("L", [1, 13, 64, 1001, 1024, 2048, 3000])
def test_n3_fast_kernel_vs_oracle(orc, K, L):
    """Reference arithmetic (U8 flag) and exact metrics both take the fast kernel and equal the
    oracle's restatements bit for bit, garbage high bits included (odd and even T at K = 9)."""
    g, kname = N3[K]
    F = 37 if K == 7 else 21
    for p, seed in ((0.0, 11), (0.04, 12), (0.09, 13), (0.5, 14)):
        if L % 8 == 0:
            unc, rx = k1n_frames(orc, K, g, L, F, p, seed + L, garbage=(p == 0.04))
        else:
            unc, rx = None, np.random.default_rng(seed + 5 * L).integers(0, 256, (F, L + K - 1), dtype=np.uint8)
        got, kern = genk_device_kernel(K, g, rx, L, native.VTB_GENK_K1_REFERENCE_U8)
        assert kern == kname, kern
        assert (got == orc.k1n_decode(K, g, rx, L)).all(), (K, L, p)
        exact, kern = genk_device_kernel(K, g, rx, L, 0)
        assert kern == kname, kern
        assert (exact == orc.genk_decode(1, K, g, rx, L)).all(), (K, L, p)
        if unc is not None and p == 0.0:
            assert (got == unc).all()


@pytest.mark.parametrize("K,g", [(7, (0o133, 0o171, 0o165)), (7, (0o117, 0o127, 0o155)), (7, (0o132, 0o171, 0o165)),
                                 (7, (0o133, 0o070, 0o165)), (9, (0o557, 0o663, 0o711)), (9, (0o556, 0o663, 0o711))])
def test_n3_generators(orc, K, g, monkeypatch):
    """Any generator set in the reference's arithmetic (the upper predecessor's metric n - e, whatever
    the taps: viterbiDecoderButterflyk1.c:104-107) on the fast kernel; exact metrics stay on the
    general kernel unless every generator taps both ends (n - e is then the true Hamming metric)."""
    kname = N3[K][1]
    L = 1024
    unc, rx = k1n_frames(orc, K, g, L, 64, 0.07, 21)
    got, kern = genk_device_kernel(K, g, rx, L, native.VTB_GENK_K1_REFERENCE_U8)
    assert kern == kname
    assert (got == orc.k1n_decode(K, g, rx, L)).all()
    ref, kern = genk_device_kernel(K, g, rx, L, native.VTB_GENK_K1_REFERENCE_U8, monkeypatch, force_genk=True)
    assert kern == "genk" and (ref == got).all()
    exact, kern = genk_device_kernel(K, g, rx, L, 0)
    ends = all((x >> (K - 1)) & 1 and x & 1 for x in g)
    assert kern == (kname if ends else "genk"), (g, kern)
    assert (exact == orc.genk_decode(1, K, g, rx, L)).all()


@pytest.mark.parametrize("K", [7, 9])
def test_n3_full_batch_and_persistent_grid(orc, K):
    """4,096 x 1,024 frames, 1,001 (one launch round) and a batch past what the CUs hold at once
    (the persistent loop) against the oracle, every frame; an odd frame count and a strided input."""
    g, kname = N3[K]
    L = 1024
    unc, rx = k1n_frames(orc, K, g, L, 4096, 0.06, 31)
    got, kern = genk_device_kernel(K, g, rx, L, native.VTB_GENK_K1_REFERENCE_U8)
    assert kern in (kname, kname + "_loop")
    assert (got == orc.k1n_decode(K, g, rx, L)).all()
    got, kern = genk_device_kernel(K, g, rx[:1001], L, native.VTB_GENK_K1_REFERENCE_U8)
    assert kern == kname
    assert (got == orc.k1n_decode(K, g, rx[:1001], L)).all()
    big_unc, big = k1n_frames(orc, K, g, L, 2 * 8 * 256 * 2 + 3, 0.05, 32)
    got, kern = genk_device_kernel(K, g, big, L, native.VTB_GENK_K1_REFERENCE_U8)
    assert kern == kname + "_loop" or (K == 9 and kern == kname)  # (K = 9: the CUs may hold the batch)
    assert (got == orc.k1n_decode(K, g, big, L)).all()
    # strided rows: the frames inside a wider buffer
    wide = np.zeros((65, big.shape[1] + 40), np.uint8)
    wide[:, :big.shape[1]] = big[:65]
    x = torch.from_numpy(wide).cuda()
    code = native.VtbGenKCode.make(1, K, g, native.VTB_GENK_K1_REFERENCE_U8)
    out = torch.zeros((65, L // 8 + 3), dtype=torch.uint8, device="cuda")
    rc = native.lib().vtb_genk_decode_device(ctypes.byref(code), L, ctypes.c_void_p(x.data_ptr()), x.stride(0),
                                             ctypes.c_void_p(out.data_ptr()), out.stride(0), 65, None)
    assert rc == 0
    torch.cuda.synchronize()
    assert (out.cpu().numpy()[:, :L // 8] == orc.k1n_decode(K, g, big[:65], L)).all()


@pytest.mark.parametrize("name", ["k7n3", "k9n3"])
def test_n3_reference_golden_on_fast_kernel(name):
    """The reference's own golden frames (tests/golden/k1n.npz) through the batch entry."""
    z = load_golden("k1n.npz")
    K, g = K1N_PARAMS[name]
    keys = sorted({k.rsplit("_", 1)[0] for k in z if k.startswith(name + "_L")})
    assert keys
    for key in keys:
        L = int(key.split("_")[1][1:])
        got, kern = genk_device_kernel(K, g, z[key + "_rx"], L, native.VTB_GENK_K1_REFERENCE_U8)
        assert kern == N3[K][1]
        assert (got == z[key + "_decoded"]).all(), key
