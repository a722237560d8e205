"""GPU: the traceback completeness guard of every kernel family (DESIGN.md 4.0 "Traceback rule",
round-5 item 1).

Every kernel traces back in verified block-parallel chains: a block is proven once it entered on
its proven successor's exit, and each verification round re-walks the failed blocks whose
successors are proven.  A chain of n blocks needs at most n - 1 re-walk rounds, and each loop is
capped (tests/test_tb_verify_model.py pins every cap against its chain length).  Round 3 shipped
wrong bits because one cap was too small and nothing noticed.  Now, after the cap, a block still
unproven never reaches the output: the frame goes to its exact slow path -- a serial walk from
the known location (the reference's own walk, /root/reference/src/viterbiDecoderButterflyk1.c:
200-256), or for split frames the unsplit pass / the list kernel.

VTB_DEBUG bit 17 forces the guards: every chain with a block not known from the frame end skips
its checks and re-walks and takes the slow path, whatever the input.  For each family this
test checks, against the oracle, bit for bit:
* with the cap: the output is exact AND the guard fired (the testing counter,
  vtb_debug_set_guard_counter, is > 0) -- the slow path ran and is exact;
* without it (the shipped caps): the output is exact and the guard never fired on the same
  pure-noise frames -- the caps are sufficient.
"""
import ctypes

import numpy as np
import pytest

from helpers import CODES, GENK_CODES, K1N_PARAMS, Oracle, genk_frames, random_frames

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from convolutionalencdec_amd import ConvCode, GenKDecoder, ViterbiDecoder, ViterbiStream, native  # noqa: E402

CAP = 1 << 17       # VTB_DEBUG: every verified chain takes the completeness guard's slow path
NO_SPLIT = 1 << 8   # VTB_DEBUG: never split frames across the halves of a wave
SEG_OFF = 1 << 10   # VTB_DEBUG: no single-frame SEG kernel
K9_PAIR = 1 << 18   # VTB_DEBUG: K=9 frames on the pair kernel (not one frame per wave)
GEN_GS = 1 << 19    # VTB_DEBUG: the generic kernel's global-survivor variant at every length
GEN_LDS = 1 << 20   # VTB_DEBUG: the generic kernel's LDS variant wherever it fits
GUARD_CODES = {**CODES, 3: (0o7, 0o5), 4: (0o15, 0o17), 6: (0o53, 0o75), 8: (0o247, 0o371)}


@pytest.fixture(scope="module")
def orc():
    return Oracle()


@pytest.fixture(scope="module", autouse=True)
def gpu_present():
    if not torch.cuda.is_available() or native.lib().vtb_device_count() < 1:
        pytest.fail("no gfx950 GPU visible to the C ABI (GPU tests must not silently pass)")


@pytest.fixture
def counter():
    c = torch.zeros(1, dtype=torch.int32, device="cuda")
    native.set_guard_counter(c.data_ptr())
    yield c
    torch.cuda.synchronize()
    native.set_guard_counter(0)


def _noisy(orc, K, L, F, soft, seed, g=None):
    """Half pure-noise frames (paths do not merge within the walk warm-up), half at moderate
    noise (some blocks verify in the first round, others need re-walks)."""
    h = F // 2
    if soft:
        _, a = random_frames(orc, K, L, h, 0.0, seed, soft=True, sigma=4.0, g=g)
        _, b = random_frames(orc, K, L, F - h, 0.0, seed + 1, soft=True, sigma=0.9, g=g)
    else:
        _, a = random_frames(orc, K, L, h, 0.5, seed, g=g)
        _, b = random_frames(orc, K, L, F - h, 0.09, seed + 1, g=g)
    return np.ascontiguousarray(np.concatenate([a, b]).reshape(F, -1))


def _set_env(monkeypatch, dbg, kernel):
    monkeypatch.setenv("VTB_DEBUG", str(dbg))
    if kernel:
        monkeypatch.setenv("VTB_KERNEL", kernel)
    else:
        monkeypatch.delenv("VTB_KERNEL", raising=False)


def _check(counter, got, want, capped, what, reachable=True):
    torch.cuda.synchronize()
    hits = int(counter.item())
    bad = np.flatnonzero((np.asarray(got) != np.asarray(want)).reshape(len(want), -1).any(axis=1))
    assert bad.size == 0, f"{what}: {bad.size} frames differ from the oracle (first {bad[:5].tolist()}), guard hits {hits}"
    if not capped:
        assert hits == 0, f"{what}: the guard fired {hits} times at the shipped round caps (a cap is too small)"
    elif reachable:
        assert hits > 0, f"{what}: the capped verification never left a chain unproven (test does not exercise the guard)"
    return hits


# kernel instances whose completeness guard counts once per frame (the K=7 pair kernels count once
# per wave)
PER_FRAME_GUARD = ("k9", "k9_loop", "k9s", "lds_path", "lds_path_gs")

# (id, K, L, frames, soft, extra VTB_DEBUG bits, VTB_KERNEL, expected kernel instance)
FRAME_CASES = [
    ("k7_lds_soft", 7, 1024, 64, True, NO_SPLIT, None, "k7_lds"),
    ("k7_lds_hard", 7, 1000, 63, False, NO_SPLIT, None, "k7_lds"),
    ("k7_lds_loop", 7, 512, 8192, False, 0, None, "k7_lds_loop"),
    ("k7_lds_split_soft", 7, 1024, 9, True, 0, None, "k7_lds_split"),
    ("k7_lds_split_hard", 7, 2900, 5, False, 0, None, "k7_lds_split"),
    ("k7_split_loop_soft", 7, 2048, 65, True, 0, "k7s", "k7_split_loop"),
    ("k7_split_loop_hard", 7, 2000, 64, False, 0, "k7s", "k7_split_loop"),
    ("k7_global_soft", 7, 1024, 64, True, 0, "gws", "k7_global"),
    ("k7_global_hard_hybrid", 7, 1024, 64, False, 0, "gws", "k7_global"),
    ("k7_global_loop", 7, 512, 8192, True, 0, "gws", "k7_global_loop"),
    ("k9s_soft", 9, 1024, 64, True, 0, None, "k9s"),
    ("k9s_hard", 9, 1001, 33, False, 0, None, "k9s"),
    ("k9s_long", 9, 16383, 5, True, 0, None, "k9s"),
    ("k9_soft", 9, 1024, 64, True, K9_PAIR, None, "k9"),
    ("k9_hard", 9, 1001, 33, False, K9_PAIR, None, "k9"),
    ("k9_loop", 9, 512, 24576, False, 0, None, "k9_loop"),
    ("lds_path_k3", 3, 3000, 64, False, GEN_LDS, None, "lds_path"),
    ("lds_path_k4_soft", 4, 2500, 16, True, GEN_LDS, None, "lds_path"),
    ("lds_path_k6", 6, 1000, 8, False, GEN_LDS, None, "lds_path"),
    ("lds_path_k8_soft", 8, 600, 3, True, GEN_LDS, None, "lds_path"),
    ("lds_path_gs_k5", 5, 16384, 9, False, 0, None, "lds_path_gs"),
    ("lds_path_gs_k3", 3, 9000, 40, False, 0, None, "lds_path_gs"),
    ("lds_path_gs_k5_soft", 5, 3000, 17, True, GEN_GS, None, "lds_path_gs"),
    ("lds_path_gs_k7_soft", 7, 2000, 16, True, GEN_GS, "lds", "lds_path_gs"),
    ("lds_path_gs_k9", 9, 1500, 5, False, GEN_GS, "lds", "lds_path_gs"),
]


@pytest.mark.parametrize("capped", [True, False], ids=["forced", "shipped"])
@pytest.mark.parametrize("case", FRAME_CASES, ids=[c[0] for c in FRAME_CASES])
def test_frame_kernels(orc, counter, monkeypatch, case, capped):
    name, K, L, F, soft, extra, kernel, inst = case
    g = GUARD_CODES[K]
    x = _noisy(orc, K, L, F, soft, 700 + K + L, g)
    want = orc.decode(K, g, x, L, soft=soft, threads=16)
    _set_env(monkeypatch, (CAP if capped else 0) | extra, kernel)
    d = ViterbiDecoder(ConvCode(K, g), frame_bits=L, soft=soft)
    got = d.decode_device(torch.from_numpy(x).cuda()).cpu().numpy()
    assert native.last_kernel() == inst, native.last_kernel()
    hits = _check(counter, got, want, capped, name)
    if capped and inst in PER_FRAME_GUARD:
        # one count per real frame: every frame here has blocks not known from its end, and a
        # lone last frame of a pair kernel has no frame B to walk (odd F counted F + 1)
        assert hits == F, (name, hits, F)


@pytest.mark.parametrize("capped", [True, False], ids=["forced", "shipped"])
@pytest.mark.parametrize("K,L,soft", [(7, 2048, True), (7, 3000, False), (9, 2048, True), (9, 1024, False),
                                      (3, 3000, True), (5, 2048, False), (8, 2048, True)])
def test_single_frame_seg(orc, counter, monkeypatch, K, L, soft, capped):
    """vtb_decode_frame_sync: the SEG kernels (one chain of up to 64 blocks over the frame's
    segments) and, where the segments do not converge, the frame kernels."""
    frames = []
    # a spread of noise levels: the SEG kernel decodes a frame only if its segments' metrics
    # converge at every boundary, and its own guard fires only on such a frame whose traceback
    # blocks did not all verify on their first walk
    g = GUARD_CODES[K]
    for i, (sigma, p) in enumerate(zip((0.7, 0.8, 0.9, 1.0, 1.1, 1.2, 1.3, 1.4, 1.6, 4.0),
                                       (0.05, 0.06, 0.07, 0.08, 0.09, 0.10, 0.11, 0.12, 0.14, 0.5))):
        if soft:
            _, x = random_frames(orc, K, L, 2, 0.0, 40 + i, soft=True, sigma=sigma, g=g)
        else:
            _, x = random_frames(orc, K, L, 2, p, 40 + i, g=g)
        frames.append(np.ascontiguousarray(x.reshape(2, -1)))
    x = np.concatenate(frames)
    want = orc.decode(K, g, x, L, soft=soft, threads=16)
    _set_env(monkeypatch, CAP if capped else 0, None)
    d = ViterbiDecoder(ConvCode(K, g), frame_bits=L, soft=soft)
    got, seg_frames, seg_guarded = [], 0, 0
    for r in x:
        st0 = (ctypes.c_ulonglong * 3)()
        native.lib().vtb_debug_seg_stats(st0)
        h0 = int(counter.item())
        got.append(d.decode_frame(r))
        st1 = (ctypes.c_ulonglong * 3)()
        native.lib().vtb_debug_seg_stats(st1)
        h1 = int(counter.item())
        # a call in which a SEG launch decoded the frame (status 1) ran no frame kernel, so a
        # guard hit in it is a SEG kernel's own
        if st1[0] > st0[0]:
            seg_frames += 1
            seg_guarded += h1 > h0
    got = np.stack(got)
    assert seg_frames > 0, "no frame decoded by the SEG kernel"
    if capped:
        assert seg_guarded > 0, "the SEG kernel's own guard never fired"
    _check(counter, got, want, capped, f"seg K={K} L={L} soft={soft}")


@pytest.mark.parametrize("capped", [True, False], ids=["forced", "shipped"])
@pytest.mark.parametrize("K,soft,gen", [(7, True, False), (7, False, False), (9, True, False), (9, False, False),
                                        (5, False, True), (7, True, True), (9, False, True)])
def test_streams(orc, counter, monkeypatch, K, soft, gen, capped):
    """vtb_stream_decode (K = 7 / K = 9 stream kernels, the generic stream kernel): a frame in
    three calls, the last one emitting the unmerged remainder in verified chains."""
    L, F = 1500, 6
    x = _noisy(orc, K, L, F, soft, 900 + K)
    want = np.unpackbits(orc.decode(K, CODES[K], x, L, soft=soft, threads=16), axis=1)[:, :L]
    _set_env(monkeypatch, CAP if capped else 0, "lds" if gen and K in (7, 9) else None)
    vs = ViterbiStream(ConvCode(K, CODES[K]), streams=F, soft=soft)
    sb = 2 if soft else 1
    xd = torch.from_numpy(x).cuda()
    T = L + K - 1
    got = [[] for _ in range(F)]
    for lo, hi, last in ((0, 500, False), (500, 1100, False), (1100, T, True)):
        out, nb = vs.push(xd[:, lo * sb:hi * sb].contiguous(), last=last)
        out, nb = out.cpu().numpy(), nb.cpu().numpy()
        for f in range(F):
            assert nb[f] >= 0
            if nb[f]:
                got[f].append(np.unpackbits(out[f])[:nb[f]])
    got = np.stack([np.concatenate(g) for g in got])
    _check(counter, got, want, capped, f"stream K={K} soft={soft} gen={gen}")


@pytest.mark.parametrize("capped", [True, False], ids=["forced", "shipped"])
@pytest.mark.parametrize("which", ["genk_k2", "genk_k2_K5", "k7_lds_n3", "k9_n3"])
def test_general_k(orc, counter, monkeypatch, which, capped):
    """vtb_genk_decode_device: the general-k kernel (one chain of up to 64 blocks over the
    frame's boundaries) and the rate-1/3 K=7 / K=9 fast kernels."""
    _set_env(monkeypatch, CAP if capped else 0, None)
    if which.startswith("genk"):
        k, K, g = GENK_CODES[0] if which == "genk_k2" else GENK_CODES[3]  # 64 / 256 states
        L, F = 1536, 12
        _, a = genk_frames(orc, k, K, g, L, F // 2, 0.5, 31)
        _, b = genk_frames(orc, k, K, g, L, F - F // 2, 0.05, 32)
        rx = np.ascontiguousarray(np.concatenate([a, b]))
        want = orc.genk_decode(k, K, g, rx, L)
        got = GenKDecoder(k, K, g, L).decode_device(torch.from_numpy(rx).cuda()).cpu().numpy()
        assert native.last_kernel() == "genk"
    else:
        K = 7 if which == "k7_lds_n3" else 9
        g = K1N_PARAMS["k7n3" if K == 7 else "k9n3"][1]
        L, F = 1024, 24
        _, a = genk_frames(orc, 1, K, g, L, F // 2, 0.5, 33)
        _, b = genk_frames(orc, 1, K, g, L, F - F // 2, 0.06, 34)
        rx = np.ascontiguousarray(np.concatenate([a, b]))
        want = orc.genk_decode(1, K, g, rx, L)
        got = GenKDecoder(1, K, g, L).decode_device(torch.from_numpy(rx).cuda()).cpu().numpy()
        assert native.last_kernel() == which
    _check(counter, got, want, capped, which)


# ---- random batches with every guard forced (the fuzz family of tests/test_gpu_fuzz.py) ----

from test_gpu_fuzz import _cases as _fuzz_cases  # noqa: E402
from test_gpu_fuzz import test_random_case_vs_oracle as _fuzz_case  # noqa: E402


@pytest.mark.parametrize("case", _fuzz_cases(48, 20261105),
                         ids=lambda c: f"{c[0]}-K{c[1]}-L{c[2]}-F{c[3]}-{'soft' if c[4] else 'hard'}")
def test_random_batches_forced(orc, counter, monkeypatch, case):
    """48 seeded random batches (K = 3..9, any length, 1 to 9,001 frames, clean to pure noise,
    strided buffers) with every completeness guard forced: still bit-exact against the oracle.
    (The whole fuzz suite with VTB_DEBUG=131072: profiles/r05/final/fuzz/.)"""
    monkeypatch.setenv("VTB_DEBUG", str(CAP))
    monkeypatch.delenv("VTB_KERNEL", raising=False)
    _fuzz_case(orc, case)
