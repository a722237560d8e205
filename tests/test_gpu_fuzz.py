"""GPU: seeded random sweep over the decoder's code paths -- K (generic path K=3/5, K=7 LDS /
global-survivor / persistent / split-frame kernels, K=9), frame length, batch size (odd counts,
single frames, batches past one launch round), hard and soft input, clean to pure-noise
channels, device and strided buffers -- each case against the oracle, bit for bit."""
import os

import numpy as np
import pytest

from helpers import CODES, Oracle, random_frames

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from convolutionalencdec_amd import ConvCode, ViterbiDecoder, native  # noqa: E402

THREADS = min(16, os.cpu_count() or 1)
K3 = (0b111, 0b101)
FUZZ_CODES = {3: K3, 4: (0o15, 0o17), 5: CODES[5], 6: (0o53, 0o75), 7: CODES[7], 8: (0o247, 0o371), 9: CODES[9]}


@pytest.fixture(scope="module")
def orc():
    return Oracle()


@pytest.fixture(scope="module", autouse=True)
def gpu_present():
    if not torch.cuda.is_available() or native.lib().vtb_device_count() < 1:
        pytest.fail("no gfx950 GPU visible to the C ABI (GPU tests must not silently pass)")


# VTB_FUZZ_N / VTB_FUZZ_SEED: a longer sweep on demand (the default is the committed sweep)
FUZZ_N = int(os.environ.get("VTB_FUZZ_N", "0"))
FUZZ_SEED = int(os.environ.get("VTB_FUZZ_SEED", "0"))


def _cases(n=FUZZ_N or 128, seed=FUZZ_SEED or 20261016):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        K = int(rng.choice([3, 4, 5, 6, 7, 7, 7, 7, 8, 9, 9]))
        # half the cases at the listed lengths (mode limits, up to the reference's 16,384), half at
        # any length (one in four of those up to 16,384): the split and segment geometries depend
        # on T modulo 48 and 96 (a floored split point once left the second half of a frame one
        # step short at T = 1 mod 96), the generic kernel's variant on T and the batch (round 6)
        if rng.integers(0, 2):
            L = int(rng.choice([1, 8, 57, 200, 234, 500, 1024, 1519, 2048, 3000, 4100, 9000, 16383, 16384]))
        else:
            L = int(rng.integers(1, 16385 if rng.integers(0, 4) == 0 else 4200))
        F = int(rng.choice([1, 2, 3, 65, 257, 1000, 2049, 4097, 9001]))
        while F * L > 12_000_000 or (K == 9 and F * L > 3_000_000):
            F = max(1, F // 3)
        soft = bool(rng.integers(0, 2))
        noise = float(rng.choice([0.0, 0.03, 0.07, 0.5]))
        strided = bool(rng.integers(0, 4) == 0)
        out.append((i, K, L, F, soft, noise, strided))
    return out


@pytest.mark.parametrize("case", _cases(), ids=lambda c: f"{c[0]}-K{c[1]}-L{c[2]}-F{c[3]}-{'soft' if c[4] else 'hard'}")
def test_random_case_vs_oracle(orc, case):
    i, K, L, F, soft, noise, strided = case
    g = FUZZ_CODES[K]
    if soft:
        sigma = {0.0: 0.3, 0.03: 0.56, 0.07: 0.7, 0.5: 4.0}[noise]
        unc, x = random_frames(orc, K, L, F, 0.0, 1000 + i, soft=True, sigma=sigma, g=g)
    else:
        unc, x = random_frames(orc, K, L, F, noise, 1000 + i, g=g)
    x = np.ascontiguousarray(x).reshape(F, -1)
    want = orc.decode(K, g, x, L, soft=soft, threads=THREADS)
    d = ViterbiDecoder(ConvCode(K, g), frame_bits=L, soft=soft)
    if strided:  # rows inside wider device buffers, output rows wider than the frame
        pad_in, pad_out = 37, 5
        xi = torch.zeros((F, x.shape[1] + pad_in), dtype=torch.uint8, device="cuda")
        xi[:, :x.shape[1]] = torch.from_numpy(x).cuda()
        ob = (L + 7) // 8
        out = torch.full((F, ob + pad_out), 0xA5, dtype=torch.uint8, device="cuda")
        native.check(native.lib().vtb_decode_device(d._plan, xi.data_ptr(), xi.stride(0), out.data_ptr(), out.stride(0),
                                                    F, None), "vtb_decode_device")
        torch.cuda.synchronize()
        got = out.cpu().numpy()
        assert (got[:, ob:] == 0xA5).all(), "wrote past the output row"
        got = got[:, :ob]
    else:
        got = d.decode_device(torch.from_numpy(x).cuda()).cpu().numpy()
    bad = np.flatnonzero((got != want).any(axis=1))
    assert bad.size == 0, (case, bad.size, bad[:8])


def _frame_cases(n=FUZZ_N or 72, seed=(FUZZ_SEED + 1) if FUZZ_SEED else 20261017):
    """K = 7, 9 (their SEG kernels) two cases in three; every other K (the generic segments,
    round 6: K = 3..6 on one workgroup, K = 6, 8 over four) the third."""
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        K = (7, 9, int(rng.choice([3, 4, 5, 6, 8])))[i % 3]
        soft = bool(rng.integers(0, 2))
        L = int(rng.integers(1, 4090 if soft else 8100))
        if K == 9 and L > 12000:
            L = 12000
        noise = float(rng.choice([0.0, 0.03, 0.07, 0.5]))
        out.append((i, L, soft, noise, K))
    return out


@pytest.mark.parametrize("case", _frame_cases(),
                         ids=lambda c: f"{c[0]}-K{c[4]}-L{c[1]}-{'soft' if c[2] else 'hard'}-p{c[3]}")
def test_single_frame_path_vs_oracle(orc, case, monkeypatch):
    """vtb_decode_frame_sync (the segmented single-frame kernels, K=7 on one workgroup, K=9
    over several, the generic segments for every other K, or the frame-kernel fallback when a
    segment has not converged) at random frame lengths and noise levels."""
    monkeypatch.delenv("VTB_KERNEL", raising=False)
    i, L, soft, noise, K = case
    g = FUZZ_CODES[K]
    if soft:
        sigma = {0.0: 0.3, 0.03: 0.56, 0.07: 0.7, 0.5: 4.0}[noise]
        unc, x = random_frames(orc, K, L, 3, 0.0, 5000 + i, soft=True, sigma=sigma, g=g)
    else:
        unc, x = random_frames(orc, K, L, 3, noise, 5000 + i, g=g)
    x = np.ascontiguousarray(x).reshape(3, -1)
    want = orc.decode(K, g, x, L, soft=soft, threads=THREADS)
    d = ViterbiDecoder(ConvCode(K, g), frame_bits=L, soft=soft)
    got = np.stack([d.decode_frame(r) for r in x])
    assert (got == want).all(), case


@pytest.mark.parametrize("L", [1100, 2047, 2048, 3001, 6000, 9999, 16384])
@pytest.mark.parametrize("noise", [0.04, 0.5])
def test_global_survivor_variant_hard_hybrid(orc, L, noise, monkeypatch):
    """The K=7 global-survivor variant on hard input keeps its newest steps' words in LDS and
    walks LDS and global blocks together; forced for every frame length."""
    monkeypatch.setenv("VTB_KERNEL", "gws")
    F = 129
    unc, x = random_frames(orc, 7, L, F, noise, 7000 + L)
    want = orc.decode(7, CODES[7], x, L, threads=THREADS)
    got = ViterbiDecoder(ConvCode(7, CODES[7]), frame_bits=L).decode_device(torch.from_numpy(x).cuda()).cpu().numpy()
    assert (got == want).all()


def _stream_cases(n=(FUZZ_N // 8) or 24, seed=(FUZZ_SEED + 2) if FUZZ_SEED else 20261018):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        K = int(rng.choice([7, 7, 9, 3, 4, 5, 6, 8]))  # (K != 7, 9: the generic stream kernel)
        soft = bool(rng.integers(0, 2))
        L = int(rng.integers(1, 6000))
        F = int(rng.integers(1, 10))
        noise = float(rng.choice([0.0, 0.03, 0.07, 0.5]))
        out.append((i, K, L, F, soft, noise))
    return out


@pytest.mark.parametrize("case", _stream_cases(),
                         ids=lambda c: f"{c[0]}-K{c[1]}-L{c[2]}-F{c[3]}-{'soft' if c[4] else 'hard'}-p{c[5]}")
def test_stream_random_chunking_vs_oracle(orc, case):
    """The streaming decoder (vtb_stream_*: K=7, K=9 and the generic stream kernel, whose calls
    start at any trellis phase) at random frame lengths, stream counts, noise levels and
    chunkings (calls of 0 to 1,200 segments, two frames per object):
    the bits each stream emits over a frame's calls, concatenated, equal the oracle's
    whole-frame decode."""
    from convolutionalencdec_amd import ViterbiStream

    i, K, L, F, soft, noise = case
    rng = np.random.default_rng(4000 + i)
    g = FUZZ_CODES[K]
    sb = 2 if soft else 1
    T = L + K - 1
    vs = ViterbiStream(ConvCode(K, g), streams=F, soft=soft)
    for frame in range(2):
        if soft:
            sigma = {0.0: 0.3, 0.03: 0.56, 0.07: 0.7, 0.5: 4.0}[noise]
            unc, x = random_frames(orc, K, L, F, 0.0, 3000 + 2 * i + frame, soft=True, sigma=sigma, g=g)
        else:
            unc, x = random_frames(orc, K, L, F, noise, 3000 + 2 * i + frame, g=g)
        x = np.ascontiguousarray(x).reshape(F, -1)
        want = np.unpackbits(orc.decode(K, g, x, L, soft=soft, threads=THREADS), axis=1)[:, :L]
        xd = torch.from_numpy(x).cuda()
        got = [[] for _ in range(F)]
        pos = 0
        while True:
            c = int(min(T - pos, rng.integers(0, 1201)))
            last = pos + c == T
            out, nb = vs.push(xd[:, pos * sb:(pos + c) * sb] if c else None, last=last)
            pos += c
            out, nb = out.cpu().numpy(), nb.cpu().numpy()
            assert (nb >= 0).all(), (case, frame, pos)
            for f in range(F):
                if nb[f] > 0:
                    got[f].append(np.unpackbits(out[f])[:nb[f]])
            if last:
                break
        for f in range(F):
            bits = np.concatenate(got[f]) if got[f] else np.zeros(0, np.uint8)
            assert bits.size == L and (bits == want[f]).all(), (case, frame, f)


def _genk_cases(n=(FUZZ_N // 8) or 16, seed=(FUZZ_SEED + 3) if FUZZ_SEED else 20261019):
    from helpers import GENK_CODES

    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        c = int(rng.integers(0, len(GENK_CODES)))
        k = GENK_CODES[c][0]
        unit = 8 * k // np.gcd(8, k)  # info bits: a multiple of 8 and of k
        L = unit * int(rng.integers(1, 3000 // unit + 1))
        F = int(rng.choice([1, 2, 3, 17, 64, 257, 1000]))
        p = float(rng.choice([0.0, 0.02, 0.08, 0.5]))
        out.append((i, c, L, F, p))
    return out


@pytest.mark.parametrize("case", _genk_cases(), ids=lambda c: f"{c[0]}-code{c[1]}-L{c[2]}-F{c[3]}-p{c[4]}")
def test_genk_random_vs_oracle(orc, case):
    """The general rate-k/n decoder (vtb_genk_decode_device) at random codes of the test set,
    frame lengths, batch sizes and BSC noise, against oracle_genk_decode."""
    from helpers import GENK_CODES, genk_frames

    from convolutionalencdec_amd import GenKDecoder

    i, c, L, F, p = case
    k, K, g = GENK_CODES[c]
    unc, coded = genk_frames(orc, k, K, g, L, F, p, 6000 + i)
    want = orc.genk_decode(k, K, g, coded, L)
    got = GenKDecoder(k, K, g, L).decode_device(torch.from_numpy(coded).cuda()).cpu().numpy()
    bad = np.flatnonzero((got != want).any(axis=1))
    assert bad.size == 0, (case, bad.size, bad[:8])


def _generator_cases(n=40, seed=20261017):
    """Every constraint length of the batch decoder (K = 3..9: the generic LDS path at K = 3-6
    and 8, the K=7 and K=9 kernels) with random generator pairs that have both end taps (the
    reference's symmetric-butterfly requirement, viterbiDecoder.c:17-25)."""
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        K = int(rng.integers(3, 10))
        g = tuple(int(1 | (1 << (K - 1)) | (int(rng.integers(0, 1 << K)) & ((1 << (K - 1)) - 2))) for _ in range(2))
        L = int(rng.integers(1, 2100))
        F = int(rng.choice([1, 3, 64, 255, 700]))
        soft = bool(rng.integers(0, 2))
        noise = float(rng.choice([0.0, 0.05, 0.5]))
        out.append((i, K, g, L, F, soft, noise))
    return out


@pytest.mark.parametrize("case", _generator_cases(),
                         ids=lambda c: f"{c[0]}-K{c[1]}-g{c[2][0]:o}_{c[2][1]:o}-L{c[3]}-F{c[4]}-{'soft' if c[5] else 'hard'}")
def test_random_generators_vs_oracle(orc, case):
    i, K, g, L, F, soft, noise = case
    if soft:
        sigma = {0.0: 0.3, 0.05: 0.6, 0.5: 4.0}[noise]
        unc, x = random_frames(orc, K, L, F, 0.0, 5000 + i, soft=True, sigma=sigma, g=g)
    else:
        unc, x = random_frames(orc, K, L, F, noise, 5000 + i, g=g)
    x = np.ascontiguousarray(x).reshape(F, -1)
    want = orc.decode(K, g, x, L, soft=soft, threads=THREADS)
    got = ViterbiDecoder(ConvCode(K, g), frame_bits=L, soft=soft).decode_device(torch.from_numpy(x).cuda()).cpu().numpy()
    bad = np.flatnonzero((got != want).any(axis=1))
    assert bad.size == 0, (case, bad.size, bad[:8])
    if noise == 0.0:
        assert (got == unc).all()
