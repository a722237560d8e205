"""GPU parity of the K=9 streaming decoder (vtb_stream_* on a 256-state code, the K=9 kernel's
STREAM variant): for any chunking, the bits a stream emits over a frame's calls, concatenated,
equal the whole-frame decode (the oracle's, pinned to the reference's K=9 golden vectors) bit
for bit -- including odd frame lengths (the soft padding survivors are rewritten one step at a
time at last), frames past the reference's 16384-bit limit and window overflow."""
import numpy as np
import pytest

from helpers import CODES, Oracle, golden_sets, hard_to_soft, random_frames
from test_gpu_stream import push_frame, random_chunks

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from convolutionalencdec_amd import ConvCode, ViterbiDecoder, ViterbiStream, native  # noqa: E402

K = 9
CODE = ConvCode(K, CODES[K])


@pytest.fixture(scope="module")
def orc():
    return Oracle()


@pytest.fixture(scope="module", autouse=True)
def gpu_present():
    if not torch.cuda.is_available() or native.lib().vtb_device_count() < 1:
        pytest.fail("no gfx950 GPU visible to the C ABI (GPU tests must not silently pass)")


def expect_bits(orc, x_host, L, soft):
    return np.unpackbits(orc.decode(K, CODES[K], x_host, L, soft=soft), axis=1)[:, :L]


def frames_for(orc, L, F, soft, seed):
    if soft:
        return random_frames(orc, K, L, F, 0.0, seed, soft=True, sigma=0.6287)
    return random_frames(orc, K, L, F, 0.04, seed)


@pytest.mark.parametrize("soft", [False, True])
@pytest.mark.parametrize("L,F", [(1, 3), (41, 4), (42, 2), (1023, 6), (1024, 5), (5001, 5)])
def test_random_chunking_matches_whole_frame(orc, soft, L, F):
    rng = np.random.default_rng(100 * L + F + soft)
    unc, xh = frames_for(orc, L, F, soft, 7 + L)
    sb = 2 if soft else 1
    T = L + K - 1
    x = torch.from_numpy(np.ascontiguousarray(xh).reshape(F, -1)).cuda()
    vs = ViterbiStream(CODE, streams=F, soft=soft)
    want = expect_bits(orc, xh, L, soft)
    # the frame decoder agrees with the oracle on these frames
    assert (ViterbiDecoder(CODE, frame_bits=L, soft=soft).decode_host(xh) == orc.decode(K, CODES[K], xh, L, soft=soft)).all()
    for trial in range(3):  # the object restarts after each last call
        got, counts = push_frame(vs, x, sb, random_chunks(rng, T))
        for f in range(F):
            assert got[f].size == L and (got[f] == want[f]).all(), (trial, f)
        assert (counts[:-1] % 8 == 0).all() and (counts >= 0).all()


def test_golden_vectors_streamed(orc):
    """The reference's K=9 golden frames (hard and the soft bridge q = 255*bit) in 100-segment chunks."""
    for key, L, unc, rx, dec in golden_sets(K):
        F, T = rx.shape
        want = np.unpackbits(dec, axis=1)[:, :L]
        for soft in (False, True):
            xh = hard_to_soft(rx) if soft else rx
            x = torch.from_numpy(np.ascontiguousarray(xh).reshape(F, -1)).cuda()
            vs = ViterbiStream(CODE, streams=F, soft=soft)
            chunks = [100] * (T // 100) + [T % 100]
            got, _ = push_frame(vs, x, 2 if soft else 1, chunks)
            for f in range(F):
                assert (got[f] == want[f]).all(), (key, soft, f)


@pytest.mark.parametrize("soft", [False, True])
def test_frames_beyond_reference_limit(orc, soft):
    """20,001-bit frames in 2048-segment chunks; bits leave the decoder long before the end."""
    L, F = 20001, 4
    unc, xh = frames_for(orc, L, F, soft, 99)
    T = L + K - 1
    x = torch.from_numpy(np.ascontiguousarray(xh).reshape(F, -1)).cuda()
    vs = ViterbiStream(CODE, streams=F, soft=soft, window_steps=4096)
    chunks = [2048] * (T // 2048) + [T % 2048]
    got, counts = push_frame(vs, x, 2 if soft else 1, chunks)
    want = expect_bits(orc, xh, L, soft)
    for f in range(F):
        assert (got[f] == want[f]).all(), f
    assert (counts[1] >= 2048 - 512).all(), counts[1]


def test_window_overflow_is_flagged_and_recovers(orc):
    F, L = 16, 1500
    T = L + K - 1
    rng = np.random.default_rng(6)
    noise = rng.integers(0, 4, (F, T), dtype=np.uint8)
    vs = ViterbiStream(CODE, streams=F, soft=False, window_steps=96)
    got, counts = push_frame(vs, torch.from_numpy(noise).cuda(), 1, [48] * (T // 48) + [T % 48])
    lost = (counts == -1).any(axis=0)
    assert lost.any()
    want = expect_bits(orc, noise, L, False)
    for f in range(F):
        if lost[f]:
            first = int(np.argmax(counts[:, f] == -1))
            assert (counts[first:, f] == -1).all()
        else:
            assert (got[f] == want[f]).all(), f
    unc, xh = random_frames(orc, K, L, F, 0.0, 6)
    got, counts = push_frame(vs, torch.from_numpy(xh).cuda(), 1, [48] * (T // 48) + [T % 48])
    assert (counts >= 0).all()
    want = np.unpackbits(unc, axis=1)[:, :L]
    for f in range(F):
        assert (got[f] == want[f]).all(), f
