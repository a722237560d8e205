"""GPU: every frame length the reference decodes, for every k = 1 rate-1/2 code the drop-in
builds (VERDICT r5 missing #1, #2, #4).

The reference decodes frames of up to MAX_PKT_LEN_UNCODED_BITS = 16,384 information bits for
any code (/root/reference/src/viterbiDecoder.h:18,45,145; viterbiDecoderButterflyk1.c:82-263).
Here K = 7 and K = 9 have their own kernels; every other K runs the generic kernel, whose LDS
variant holds a wave's survivors and input in LDS and whose GS variant (vtb_lds_path.hip) keeps
the survivors in a global workspace -- every length up to 16,384, hard and soft.

Checked bit for bit against:
* tests/golden/lengths.npz -- the reference decoder's own outputs at L = 1, 7, 100, 1001, 4095,
  9000, 16383, 16384 (make_golden_lengths.py), through the batch C ABI (every kernel family
  that decodes the code, hard and the soft bridge q = 255*bit) and through the legacy drop-in
  libraries (include/viterbiDecoder.h, one per code configuration, with no viterbiConfigCheck
  call, as the reference harnesses may do);
* the oracle at L = 16,384 on fresh seeded hard and soft batches of every K.
"""
import ctypes
import os

import numpy as np
import pytest

from helpers import LENGTH_CODES, LENGTHS, Oracle, hard_to_soft, length_sets, legacy_layout, random_frames

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from convolutionalencdec_amd import LIB_DIR, ConvCode, ViterbiDecoder, native  # noqa: E402

SYMMETRIC = [n for n in sorted(LENGTH_CODES) if n != "k3"]
GEN_GS = 1 << 19  # VTB_DEBUG: the generic kernel's global-survivor variant at every length
GEN_LDS = 1 << 20  # VTB_DEBUG: the generic kernel's LDS variant wherever it fits one CU


@pytest.fixture(scope="module")
def orc():
    return Oracle()


@pytest.fixture(scope="module", autouse=True)
def gpu_present():
    if not torch.cuda.is_available() or native.lib().vtb_device_count() < 1:
        pytest.fail("no gfx950 GPU visible to the C ABI (GPU tests must not silently pass)")


def _families(K):
    """(VTB_KERNEL, VTB_DEBUG) settings that decode constraint length K."""
    fam = [(None, 0), ("lds", 0), ("lds", GEN_GS), ("lds", GEN_LDS)]
    if K == 7:
        fam += [("k7", 0), ("gws", 0), ("k7s", 0)]
    if K == 9:
        fam += [("k9", 0), ("k9", 1 << 18)]
    return fam


def _env(monkeypatch, kernel, dbg):
    if kernel:
        monkeypatch.setenv("VTB_KERNEL", kernel)
    else:
        monkeypatch.delenv("VTB_KERNEL", raising=False)
    monkeypatch.setenv("VTB_DEBUG", str(dbg))


def _dev(d, x):
    xd = torch.from_numpy(np.ascontiguousarray(x).reshape(x.shape[0], -1)).cuda()
    out = d.decode_device(xd)
    torch.cuda.synchronize()
    return out.cpu().numpy()


@pytest.mark.parametrize("name", SYMMETRIC)
def test_reference_lengths_every_kernel(monkeypatch, name):
    """The reference's decodes at every fixture length, every kernel family, hard and soft
    bridge, through the batch device entry point."""
    K, g = LENGTH_CODES[name]
    for kernel, dbg in _families(K):
        _env(monkeypatch, kernel, dbg)
        for key, _, K_, g_, L, unc, rx, dec in length_sets([name]):
            for soft in (False, True):
                d = ViterbiDecoder(ConvCode(K, g), frame_bits=L, soft=soft)
                x = hard_to_soft(rx) if soft else rx
                try:
                    got = _dev(d, x)
                except native.VtbError:
                    # only the forced K=7 LDS-resident kernel has a shape window (its LDS
                    # capacity); every other family must take every length
                    assert kernel == "k7", (key, kernel, soft)
                    d.close()
                    continue
                assert (got == dec).all(), (key, kernel, dbg, soft, native.last_kernel())
                if kernel == "lds" and dbg == GEN_GS:
                    assert native.last_kernel() == "lds_path_gs", (key, native.last_kernel())
                d.close()


@pytest.mark.parametrize("soft", [False, True])
@pytest.mark.parametrize("name", SYMMETRIC)
def test_max_length_vs_oracle(orc, name, soft):
    """L = 16,384 (and 16,383) batches of every K on the library's own kernel choice, against
    the oracle: clean frames decode to the payload, noisy and pure-noise frames to the oracle."""
    K, g = LENGTH_CODES[name]
    for L in (16383, 16384):
        d = ViterbiDecoder(ConvCode(K, g), frame_bits=L, soft=soft)
        for noise, seed in ((0.0, 1), (0.05, 2), (0.5, 3)):
            F = 37
            if soft:
                sigma = (0.3, 0.75, 4.0)[seed - 1]
                unc, x = random_frames(orc, K, L, F, 0.0, 100 * K + seed + L, soft=True, sigma=sigma, g=g)
            else:
                unc, x = random_frames(orc, K, L, F, noise, 100 * K + seed + L, g=g)
            want = orc.decode(K, g, x, L, soft=soft, threads=16)
            got = _dev(d, x)
            bad = np.flatnonzero((got != want).any(axis=1))
            assert bad.size == 0, (name, L, soft, seed, native.last_kernel(), bad[:8])
            if seed == 1:
                assert (got == unc).all()
        if K not in (7, 9):
            assert native.last_kernel() == "lds_path_gs", native.last_kernel()


@pytest.mark.parametrize("name", [n for n in SYMMETRIC if LENGTH_CODES[n][0] not in (7, 9)])
def test_large_batch_long_frames(orc, name):
    """A batch whose survivor words exceed the GS variant's workspace cap (1 GiB: the batch runs
    as several launches over the one workspace): every frame against the oracle (64 distinct
    frames repeated, so each copy must equal the oracle's decode)."""
    K, g = LENGTH_CODES[name]  # (K = 7, 9: their own kernels, tests/test_gpu_parity.py)
    L = 16384
    R = 1 if K <= 7 else (1 << (K - 1)) // 64
    Fw = 64 >> (K - 1) if K <= 6 else 1  # frames per wave
    per_wave = (L + K - 1) * R * 8
    # waves per launch: 1 GiB of words, at least the 32 per CU the device holds (vtb_lds_path.hip
    # gs_waves_per_launch); just past that (K = 3: 131,139 frames, 2.1 GB of input)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    F = (max((1 << 30) // per_wave, 32 * cus) + 5) * Fw + 3
    unc, x = random_frames(orc, K, L, 64, 0.04, 5 + K, g=g)
    reps = (F + 63) // 64
    xd = torch.from_numpy(np.ascontiguousarray(x)).cuda().repeat(reps, 1)[:F].contiguous()
    d = ViterbiDecoder(ConvCode(K, g), frame_bits=L)
    out = d.decode_device(xd).cpu().numpy()
    want = orc.decode(K, g, x, L, threads=16)
    for r in range(0, reps):
        lo, hi = r * 64, min(F, (r + 1) * 64)
        assert (out[lo:hi] == want[:hi - lo]).all(), (name, F, r)


# ---------------- the legacy drop-in (include/viterbiDecoder.h) at every length ----------------

def _legacy(name):
    lib = ctypes.CDLL(os.path.join(LIB_DIR, f"libviterbi_legacy_{name}.so"))
    v = ctypes.c_void_p
    lib.viterbiInitButterflyk1.argtypes = [v]
    lib.resetViterbiDecoderHardButterflyk1.argtypes = [v]
    lib.viterbiDecoderHardButterflyk1.argtypes = [v, v, v, ctypes.c_int, ctypes.c_bool]
    return lib


def _state(K):
    size = legacy_layout(1, K, 2)["sizeof"]
    buf = np.zeros(size + 64, np.uint8)
    off = (-buf.ctypes.data) % 64
    return buf, ctypes.c_void_p(buf.ctypes.data + off)


@pytest.mark.parametrize("name", sorted(LENGTH_CODES))
def test_legacy_dropin_reference_lengths(name):
    """Each code configuration's legacy library (built from params/<name>, the harness config
    the reference would be compiled with) decodes the reference's fixtures at every length up to
    16,384 bits, with the reference's return value (:256), whole frames with last=true and --
    for the longest -- in last=false chunks first.  "k3" is handTraced's non-symmetric code
    (0b111, 0b110): viterbiConfigCheck would reject it, and the reference still decodes it with
    its butterfly arithmetic when the harness does not call the check."""
    K, g = LENGTH_CODES[name]
    lib = _legacy(name)
    buf, st = _state(K)
    lib.resetViterbiDecoderHardButterflyk1(st)
    lib.viterbiInitButterflyk1(st)
    seen = set()
    for key, _, K_, g_, L, unc, rx, dec in length_sets([name]):
        seen.add(L)
        for f in range(rx.shape[0]):
            out = np.zeros(dec.shape[1], np.uint8)
            row = np.ascontiguousarray(rx[f])
            r = lib.viterbiDecoderHardButterflyk1(st, row.ctypes.data_as(ctypes.c_void_p),
                                                  out.ctypes.data_as(ctypes.c_void_p), len(row), True)
            assert r == (L - 1) // 8 + 1, (key, r)
            assert (out == dec[f]).all(), (key, f)
        if L == 16384:
            row = np.ascontiguousarray(rx[0])
            out = np.zeros(dec.shape[1], np.uint8)
            c = 0
            while len(row) - c > 5000:
                ch = np.ascontiguousarray(row[c:c + 5000])
                assert lib.viterbiDecoderHardButterflyk1(st, ch.ctypes.data_as(ctypes.c_void_p),
                                                         out.ctypes.data_as(ctypes.c_void_p), 5000, False) == 0
                c += 5000
            rest = np.ascontiguousarray(row[c:])
            assert lib.viterbiDecoderHardButterflyk1(st, rest.ctypes.data_as(ctypes.c_void_p),
                                                     out.ctypes.data_as(ctypes.c_void_p), len(rest), True) == 2048
            assert (out == dec[0]).all(), key
    assert seen == set(LENGTHS)
