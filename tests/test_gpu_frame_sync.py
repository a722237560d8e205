"""GPU parity of the synchronous single-frame path (vtb_decode_frame_sync): K=7 frames cut
into up to eight segments decoded at once by one workgroup (k7_seg_kernel), with the frame
read from and the bytes written to host-mapped memory and completion signalled through host
memory; and K=9 frames cut into up to 32 segments over four workgroups on one XCD
(k9_seg_kernel, the last workgroup to arrive checks the boundaries and traces back).  Every frame is compared bit for bit with the oracle / the reference's golden
vectors; the path counters show that the segmented kernel decoded the clean and noisy frames
and that unconverged segments (pure-noise input) fall back to the frame kernel."""
import ctypes

import numpy as np
import pytest

from helpers import CODES, Oracle, golden_sets, hard_to_soft, random_frames

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from convolutionalencdec_amd import ConvCode, ViterbiDecoder, native  # noqa: E402


@pytest.fixture(scope="module")
def orc():
    return Oracle()


@pytest.fixture(scope="module", autouse=True)
def gpu_present():
    if not torch.cuda.is_available() or native.lib().vtb_device_count() < 1:
        pytest.fail("no gfx950 GPU visible to the C ABI (GPU tests must not silently pass)")


def seg_stats():
    out = (ctypes.c_ulonglong * 3)()
    native.lib().vtb_debug_seg_stats(out)
    return np.array(list(out), np.int64)  # [seg decoded, seg not converged, no seg kernel]


def run(dec, rx):
    return np.stack([dec.decode_frame(r) for r in rx])


def test_golden_vectors_k7(monkeypatch):
    monkeypatch.delenv("VTB_KERNEL", raising=False)
    s0 = seg_stats()
    for key, L, unc, rx, decd in golden_sets(7):
        for soft in (False, True):
            d = ViterbiDecoder(ConvCode(7, CODES[7]), frame_bits=L, soft=soft)
            x = hard_to_soft(rx) if soft else rx
            assert (run(d, x) == decd).all(), (key, soft)
    s1 = seg_stats()
    assert s1[0] > s0[0], (s0, s1)  # the segmented kernel ran (frames of T >= 240)


@pytest.mark.parametrize("L", [234, 300, 1000, 1024, 2048, 2049, 3000, 4090, 8000, 12000, 16384])
@pytest.mark.parametrize("soft", [False, True])
def test_random_vs_oracle(orc, L, soft, monkeypatch):
    monkeypatch.delenv("VTB_KERNEL", raising=False)
    F = 6
    if soft:
        unc, rx = random_frames(orc, 7, L, F, 0.0, seed=L, soft=True, sigma=0.63)  # the bench's SNR
    else:
        unc, rx = random_frames(orc, 7, L, F, 0.05, seed=L)
    want = orc.decode(7, CODES[7], rx, L, soft=soft)
    d = ViterbiDecoder(ConvCode(7, CODES[7]), frame_bits=L, soft=soft)
    s0 = seg_stats()
    got = run(d, rx)
    s1 = seg_stats()
    assert (got == want).all()
    if L <= 8000:  # (longer frames: the frame kernel where the segments' words exceed the LDS)
        assert s1[0] - s0[0] >= F // 2, (s0, s1)  # these noise levels mostly converge within the warm-up


@pytest.mark.parametrize("waves", [1, 2, 3, 4, 5, 7])
def test_fewer_waves(orc, waves, monkeypatch):
    monkeypatch.delenv("VTB_KERNEL", raising=False)
    monkeypatch.setenv("VTB_SEG_WAVES", str(waves))
    L = 2048
    unc, rx = random_frames(orc, 7, L, 4, 0.04, seed=waves)
    d = ViterbiDecoder(ConvCode(7, CODES[7]), frame_bits=L)
    s0 = seg_stats()
    assert (run(d, rx) == orc.decode(7, CODES[7], rx, L)).all()
    assert seg_stats()[0] > s0[0]


def test_pure_noise_falls_back(orc, monkeypatch):
    """p = 0.5: segment metrics do not converge within 96 steps; the frame is decoded again by
    the frame kernel, still bit-exact."""
    monkeypatch.delenv("VTB_KERNEL", raising=False)
    L = 2048
    unc, rx = random_frames(orc, 7, L, 8, 0.5, seed=5)
    d = ViterbiDecoder(ConvCode(7, CODES[7]), frame_bits=L)
    s0 = seg_stats()
    assert (run(d, rx) == orc.decode(7, CODES[7], rx, L)).all()
    s1 = seg_stats()
    assert s1[1] > s0[1]


@pytest.mark.parametrize("K", [3, 4, 5, 6, 8])
@pytest.mark.parametrize("soft", [False, True])
def test_other_k_segments(orc, K, soft, monkeypatch):
    """K without a single-frame kernel of its own: the generic kernel's segments (gen_seg_kernel,
    round 6), with a generator pair of both end taps drawn at random per K.  Short frames (too few
    steps for two segments) and frames whose segments' survivor words exceed the LDS take the batch
    kernel; everything in between the segments, bit-exact either way (their use counted on a
    standard code of each K)."""
    monkeypatch.delenv("VTB_KERNEL", raising=False)
    rng = np.random.default_rng(40 + K)
    weak = tuple(int(1 | (1 << (K - 1)) | (int(rng.integers(0, 1 << K)) & ((1 << (K - 1)) - 2))) for _ in range(2))
    std = {3: (0o7, 0o5), 4: (0o15, 0o17), 5: CODES[5], 6: (0o53, 0o75), 8: (0o247, 0o371)}[K]
    # a random end-tapped pair (often a weak code, whose segments rarely converge: parity only)
    for L in (1000,):
        unc, rx = random_frames(orc, K, L, 3, 0.03, seed=K + L, g=weak)
        d = ViterbiDecoder(ConvCode(K, weak), frame_bits=L)
        assert (run(d, rx) == orc.decode(K, weak, rx, L)).all(), (K, weak, L)
    g = std
    for L in (1, 77, 200, 1000, 2048, 5001, 12000, 16384):
        if soft:
            unc, rx = random_frames(orc, K, L, 3, 0.0, seed=K + L, soft=True, sigma=0.6, g=g)
            rx = rx.reshape(3, -1)
        else:
            unc, rx = random_frames(orc, K, L, 3, 0.03, seed=K + L, g=g)
        d = ViterbiDecoder(ConvCode(K, g), frame_bits=L, soft=soft)
        s0 = seg_stats()
        assert (run(d, rx) == orc.decode(K, g, rx, L, soft=soft)).all(), (K, g, L)
        ds = seg_stats() - s0
        if L <= 77:
            assert ds[2] == 3, (K, L, ds)  # no segments for so few steps
        elif 1000 <= L <= 5001:
            assert ds[0] >= 2, (K, L, ds)  # the segments decoded these frames
            assert native.last_kernel() in ("gen_seg", "lds_path", "lds_path_gs")


@pytest.mark.parametrize("K", [3, 5, 8])
def test_other_k_pure_noise_falls_back(orc, K, monkeypatch):
    """p = 0.5: the generic segments' metrics do not converge; the batch kernel decodes the frame
    again, bit-exact."""
    monkeypatch.delenv("VTB_KERNEL", raising=False)
    g = {3: (0o7, 0o5), 5: CODES[5], 8: (0o247, 0o371)}[K]
    L = 2048
    unc, rx = random_frames(orc, K, L, 6, 0.5, seed=7 + K, g=g)
    d = ViterbiDecoder(ConvCode(K, g), frame_bits=L)
    s0 = seg_stats()
    assert (run(d, rx) == orc.decode(K, g, rx, L)).all()
    assert seg_stats()[1] > s0[1]


def test_k9_golden_vectors(monkeypatch):
    """K = 9 single frames (k9_seg_kernel: segments over several workgroups) on the
    reference's K=9 golden frames, hard and the soft bridge."""
    monkeypatch.delenv("VTB_KERNEL", raising=False)
    s0 = seg_stats()
    for key, L, unc, rx, decd in golden_sets(9):
        for soft in (False, True):
            d = ViterbiDecoder(ConvCode(9, CODES[9]), frame_bits=L, soft=soft)
            x = hard_to_soft(rx) if soft else rx
            assert (run(d, x) == decd).all(), (key, soft)
    assert seg_stats()[0] > s0[0]


@pytest.mark.parametrize("L", [233, 240, 1000, 1023, 2048, 2049, 4000, 8001])
@pytest.mark.parametrize("soft", [False, True])
def test_k9_random_vs_oracle(orc, L, soft, monkeypatch):
    monkeypatch.delenv("VTB_KERNEL", raising=False)
    F = 4
    if soft:
        unc, rx = random_frames(orc, 9, L, F, 0.0, seed=90 + L, soft=True, sigma=0.63)
    else:
        unc, rx = random_frames(orc, 9, L, F, 0.04, seed=90 + L)
    want = orc.decode(9, CODES[9], rx, L, soft=soft)
    d = ViterbiDecoder(ConvCode(9, CODES[9]), frame_bits=L, soft=soft)
    s0 = seg_stats()
    assert (run(d, rx) == want).all()
    assert seg_stats()[0] - s0[0] >= F // 2, (s0, seg_stats())


@pytest.mark.parametrize("xcd", [0, 1])
@pytest.mark.parametrize("wgs", [1, 2, 5, 8])
def test_k9_workgroup_counts(orc, wgs, xcd, monkeypatch):
    """Other workgroup counts, and the workgroups spread over the XCDs instead of on one."""
    monkeypatch.delenv("VTB_KERNEL", raising=False)
    monkeypatch.setenv("VTB_SEG9_WGS", str(wgs))
    monkeypatch.setenv("VTB_SEG9_XCD", str(xcd))
    L = 2048
    unc, rx = random_frames(orc, 9, L, 3, 0.03, seed=wgs)
    d = ViterbiDecoder(ConvCode(9, CODES[9]), frame_bits=L)
    assert (run(d, rx) == orc.decode(9, CODES[9], rx, L)).all()


@pytest.mark.parametrize("soft", [False, True])
@pytest.mark.parametrize("wgs", [1, 2, 4, 8])
@pytest.mark.parametrize("K", [6, 8])
def test_generic_segment_workgroups(orc, K, wgs, soft, monkeypatch):
    """K = 6, 8 single frames: the generic segments on one workgroup (the LDS hand-over) and over
    2, 4 (shipped) and 8 workgroups (the workspace hand-over, the last workgroup to arrive checks
    and traces back), bit-exact against the oracle, and decoded by the segments."""
    monkeypatch.delenv("VTB_KERNEL", raising=False)
    monkeypatch.setenv("VTB_SEGG_WGS", str(wgs))
    g = {6: (0o53, 0o75), 8: (0o247, 0o371)}[K]
    for L in (1500, 2048, 4000):
        if soft:
            unc, rx = random_frames(orc, K, L, 3, 0.0, seed=K * wgs + L, soft=True, sigma=0.6, g=g)
            rx = rx.reshape(3, -1)
        else:
            unc, rx = random_frames(orc, K, L, 3, 0.02, seed=K * wgs + L, g=g)
        d = ViterbiDecoder(ConvCode(K, g), frame_bits=L, soft=soft)
        s0 = seg_stats()
        assert (run(d, rx) == orc.decode(K, g, rx, L, soft=soft)).all(), (K, wgs, L, soft)
        ds = seg_stats() - s0
        assert ds[0] >= 2 and ds[2] == 0, (K, wgs, L, soft, ds)
        assert native.last_kernel() in ("gen_seg", "lds_path_gs"), native.last_kernel()
        d.close()


def test_k9_pure_noise_falls_back(orc, monkeypatch):
    monkeypatch.delenv("VTB_KERNEL", raising=False)
    L = 2048
    unc, rx = random_frames(orc, 9, L, 4, 0.5, seed=9)
    d = ViterbiDecoder(ConvCode(9, CODES[9]), frame_bits=L)
    s0 = seg_stats()
    assert (run(d, rx) == orc.decode(9, CODES[9], rx, L)).all()
    assert seg_stats()[1] > s0[1]


@pytest.mark.parametrize("K", [7, 9])
def test_adaptive_warmup(orc, K, monkeypatch):
    """The short warm-up (48 steps) is tried first; after a miss the plan's own warm-up serves
    the next 64 calls (doubling per miss), so a noisy stretch costs one extra launch per
    backoff period, and clean frames take one launch each.  Bit-exact throughout."""
    monkeypatch.delenv("VTB_KERNEL", raising=False)
    monkeypatch.delenv("VTB_SEG_WARM", raising=False)
    monkeypatch.delenv("VTB_SEG_ADAPT", raising=False)
    L = 2048
    d = ViterbiDecoder(ConvCode(K, CODES[K]), frame_bits=L)
    unc, clean = random_frames(orc, K, L, 12, 0.0, seed=31 + K)
    s0 = seg_stats()
    assert (run(d, clean) == orc.decode(K, CODES[K], clean, L)).all()
    s1 = seg_stats()
    assert (s1 - s0).tolist() == [12, 0, 0], (s0, s1)  # one converged launch per clean frame
    unc, noise = random_frames(orc, K, L, 20, 0.5, seed=37 + K)
    assert (run(d, noise) == orc.decode(K, CODES[K], noise, L)).all()
    s2 = seg_stats()
    assert s2[1] - s1[1] <= 20 + 1, (s1, s2)  # one short-warm-up miss, then the plan's warm-up only
    assert s2[2] == s1[2]


def test_adaptive_off(orc, monkeypatch):
    monkeypatch.delenv("VTB_KERNEL", raising=False)
    monkeypatch.setenv("VTB_SEG_ADAPT", "0")
    L = 3000
    unc, rx = random_frames(orc, 7, L, 6, 0.03, seed=3)
    d = ViterbiDecoder(ConvCode(7, CODES[7]), frame_bits=L)
    assert (run(d, rx) == orc.decode(7, CODES[7], rx, L)).all()


def test_short_frames(orc, monkeypatch):
    monkeypatch.delenv("VTB_KERNEL", raising=False)
    for L in (1, 8, 100, 233):
        unc, rx = random_frames(orc, 7, L, 2, 0.05, seed=L)
        d = ViterbiDecoder(ConvCode(7, CODES[7]), frame_bits=L)
        assert (run(d, rx) == orc.decode(7, CODES[7], rx, L)).all(), L


def test_repeated_calls_one_plan(orc, monkeypatch):
    """Back-to-back calls on one plan (the speedDecode loop): each call's bytes are its own."""
    monkeypatch.delenv("VTB_KERNEL", raising=False)
    L = 2048
    unc, rx = random_frames(orc, 7, L, 16, 0.02, seed=77)
    want = orc.decode(7, CODES[7], rx, L)
    d = ViterbiDecoder(ConvCode(7, CODES[7]), frame_bits=L)
    for rep in range(3):
        for i in range(16):
            assert (d.decode_frame(rx[i]) == want[i]).all(), (rep, i)


@pytest.mark.parametrize("nthreads", [4, 12])
def test_concurrent_threads(orc, nthreads, monkeypatch):
    """Host threads decoding at once (one plan each, as the legacy API's per-thread plans):
    mixed shapes (two frame lengths, soft and hard, K=9) side by side, every frame
    bit-exact."""
    import threading

    monkeypatch.delenv("VTB_KERNEL", raising=False)
    shapes = [(7, 2048, False), (7, 2048, False), (7, 1000, True), (9, 2048, False)]
    jobs = []
    for i in range(nthreads):
        K, L, soft = shapes[i % len(shapes)]
        if soft:
            unc, rx = random_frames(orc, K, L, 24, 0.0, seed=700 + i, soft=True, sigma=0.5)
        else:
            unc, rx = random_frames(orc, K, L, 24, 0.02 if i % 3 else 0.0, seed=700 + i)
        jobs.append((K, L, soft, rx, orc.decode(K, CODES[K], rx, L, soft=soft)))
    decs = [ViterbiDecoder(ConvCode(K, CODES[K]), frame_bits=L, soft=soft) for K, L, soft, _, _ in jobs]
    for d, (K, L, soft, rx, want) in zip(decs, jobs):
        d.decode_frame(rx[0])  # plans and host-mapped buffers before the threads start
    errors = []

    def work(i):
        K, L, soft, rx, want = jobs[i]
        try:
            for rep in range(3):
                for f in range(rx.shape[0]):
                    got = decs[i].decode_frame(rx[f])
                    if not (got == want[f]).all():
                        errors.append((i, rep, f))
                        return
        except Exception as e:  # noqa: BLE001
            errors.append((i, repr(e)))

    th = [threading.Thread(target=work, args=(i,)) for i in range(nthreads)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in th)
    assert not errors, errors[:8]
