"""GPU parity of the generic streaming decoder (csrc/vtb_stream_gen.hip; vtb_stream_* for K
other than 7 and 9, and for K = 7 / 9 when VTB_KERNEL=lds), row f3 of SURVEY.md 8.

The contract is the reference's chunked protocol (viterbiDecoderHardButterflyk1 with
last=false, then last=true; src/viterbiDecoderButterflyk1.c:82-263): for any chunking, the
bits a stream emits over a frame's calls, concatenated, equal the whole-frame decode (the
oracle, pinned to the reference's golden vectors) bit for bit.  Unlike the K=7/9 kernels the
generic one decodes every segment of a call at once (no 48-step carry)."""
import numpy as np
import pytest

from helpers import CODES, Oracle, golden_sets, hard_to_soft, random_frames
from test_gpu_stream import push_frame, random_chunks

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from convolutionalencdec_amd import ConvCode, ViterbiStream, native  # noqa: E402

# symmetric rate-1/2 codes (both end taps set, viterbiDecoder.c:17-25) for every K
GCODES = {3: (0b111, 0b101), 4: (0o15, 0o17), 5: CODES[5], 6: (0o53, 0o75), 7: CODES[7], 8: (0o247, 0o371),
          9: CODES[9]}


@pytest.fixture(scope="module")
def orc():
    return Oracle()


@pytest.fixture(autouse=True)
def generic(monkeypatch):
    # K = 7 and 9 run their own kernels by default; the generic one is forced for them here
    monkeypatch.setenv("VTB_KERNEL", "lds")
    if not torch.cuda.is_available() or native.lib().vtb_device_count() < 1:
        pytest.fail("no gfx950 GPU visible to the C ABI (GPU tests must not silently pass)")


def stream_case(orc, K, L, F, soft, chunks_rng, p=0.05, sigma=0.6287, seed=0, window=0):
    g = GCODES[K]
    if soft:
        unc, xh = random_frames(orc, K, L, F, 0.0, seed, soft=True, sigma=sigma, g=g)
    else:
        unc, xh = random_frames(orc, K, L, F, p, seed, g=g)
    sb = 2 if soft else 1
    T = L + K - 1
    x = torch.from_numpy(np.ascontiguousarray(xh).reshape(F, -1)).cuda()
    vs = ViterbiStream(ConvCode(K, g), streams=F, soft=soft, window_steps=window)
    want = np.unpackbits(orc.decode(K, g, xh, L, soft=soft), axis=1)[:, :L]
    return vs, x, sb, T, want


@pytest.mark.parametrize("K", [3, 4, 5, 6, 7, 8, 9])
@pytest.mark.parametrize("soft", [False, True])
@pytest.mark.parametrize("L,F", [(1, 3), (42, 5), (1024, 9), (4000, 3)])
def test_random_chunking_matches_whole_frame(orc, K, soft, L, F):
    rng = np.random.default_rng(1000 * K + 10 * L + F + soft)
    vs, x, sb, T, want = stream_case(orc, K, L, F, soft, rng, seed=K * 100 + L)
    for trial in range(2):  # the object restarts after each last call
        got, counts = push_frame(vs, x, sb, random_chunks(rng, T))
        for f in range(F):
            assert got[f].size == L and (got[f] == want[f]).all(), (K, trial, f)
        assert (counts[:-1] % 8 == 0).all() and (counts >= 0).all()
    assert native.last_kernel() == "gen_stream"


@pytest.mark.parametrize("K", [3, 5, 8])
def test_many_streams_and_noise(orc, K):
    """More streams than one wave holds, noisy and pure-noise frames (slow merges carry
    unemitted steps across calls)."""
    rng = np.random.default_rng(K)
    for p in (0.08, 0.5):
        vs, x, sb, T, want = stream_case(orc, K, 3000, 70, False, rng, p=p, seed=int(p * 100) + K)
        got, _ = push_frame(vs, x, sb, random_chunks(rng, T, sizes=(5, 48, 400, 1000)))
        for f in range(70):
            assert (got[f] == want[f]).all(), (K, p, f)


def test_golden_vectors_streamed_k5():
    """The reference's K=5 golden frames (hard and the soft bridge q = 255*bit) in 100-segment chunks."""
    for key, L, unc, rx, dec in golden_sets(5):
        F, T = rx.shape
        want = np.unpackbits(dec, axis=1)[:, :L]
        for soft in (False, True):
            xh = hard_to_soft(rx) if soft else rx
            x = torch.from_numpy(np.ascontiguousarray(xh).reshape(F, -1)).cuda()
            vs = ViterbiStream(ConvCode(5, CODES[5]), streams=F, soft=soft)
            got, _ = push_frame(vs, x, 2 if soft else 1, [100] * (T // 100) + [T % 100])
            for f in range(F):
                assert (got[f] == want[f]).all(), (key, soft, f)


@pytest.mark.parametrize("soft", [False, True])
def test_long_frames_early_output(orc, soft):
    """30,000-bit K=5 frames (past the reference's 16384-bit limit) in 4000-segment calls: the
    bits leave the decoder long before the frame ends."""
    rng = np.random.default_rng(3)
    vs, x, sb, T, want = stream_case(orc, 5, 30000, 4, soft, rng, p=0.04, sigma=0.55, seed=31, window=8192)
    got, counts = push_frame(vs, x, sb, [4000] * (T // 4000) + [T % 4000])
    for f in range(4):
        assert (got[f] == want[f]).all(), f
    assert (counts[1] >= 4000 - 256).all(), counts[1]


def test_window_overflow_is_flagged_and_recovers(orc):
    """Pure noise with a 96-step window: a stream whose paths do not merge in time reports -1
    until last; afterwards every stream decodes the next frame."""
    K, F, L = 6, 16, 2000
    g = GCODES[K]
    T = L + K - 1
    noise = np.random.default_rng(5).integers(0, 4, (F, T), dtype=np.uint8)
    vs = ViterbiStream(ConvCode(K, g), streams=F, window_steps=96)
    got, counts = push_frame(vs, torch.from_numpy(noise).cuda(), 1, [48] * (T // 48) + [T % 48])
    lost = (counts == -1).any(axis=0)
    want = np.unpackbits(orc.decode(K, g, noise, L), axis=1)[:, :L]
    for f in range(F):
        if lost[f]:
            first = int(np.argmax(counts[:, f] == -1))
            assert (counts[first:, f] == -1).all()
        else:
            assert (got[f] == want[f]).all(), f
    unc, xh = random_frames(orc, K, L, F, 0.0, 6, g=g)
    got, counts = push_frame(vs, torch.from_numpy(xh).cuda(), 1, [48] * (T // 48) + [T % 48])
    assert (counts >= 0).all()
    for f in range(F):
        assert (got[f] == np.unpackbits(unc, axis=1)[f, :L]).all(), f
