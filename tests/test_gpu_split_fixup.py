"""GPU: the K=7 split-frame kernels and their in-wave fix-up (DESIGN.md 4.1 "Shapes", 4.2b;
PERF_LOG.md 4.2b "Round 3: the in-wave fix-up"), bit for bit against the oracle.

A split frame is decoded in one wave as two halves: A = steps [0, t1) from the reference's
start metrics, B = [t1 - warm, T) from equal metrics.  When B's metric vector at t1 is not A's
up to a constant, the fix-up re-runs B from A's metrics one chunk at a time until it matches
B's own metrics at a checkpoint; only a frame that still differs after kFix chunks takes the
slow path (the unsplit pass in `k7_lds_split`, the list kernel in `k7_split_loop`).  The
reference decodes every input exactly (/root/reference/src/viterbiDecoderButterflyk1.c:82-263),
so each path must too.

* `test_case_1366_*`: the round-3 failure (fuzz seed 1017 case 1366: K=7, L = 2,966, soft,
  sigma 4, three frames; 6 wrong bits at 85-93 of frame 1).  Root cause: the split pass chains
  up to 63 traceback blocks (frame A's nA <= 32, frame B's kB0-32..31 with kB0 = 32 + warm/48;
  62 at warm-up 96) but verified them in at most 33
  rounds, so on a pure-noise frame kept split by the fix-up frame A's first blocks left the
  loop unverified.  Pinned on the single-frame entry and the batch entry, under every fix-up
  mode.
* `test_fixup_family_vs_oracle`: a seeded family that forces the fix-up (VTB_DEBUG bit 15:
  on every split frame, converged or not) and its exhaustion (bit 16: no checkpoint ever
  matches, so every frame runs kFix fix-up chunks and then the slow path) on both instances,
  across T mod 48 / mod 96 residues, batch sizes 1, 2, 3, 65, 2,048 and the persistent C3
  shape, soft and hard input, clean to pure noise.  VTB_FIXUP_N / VTB_FIXUP_SEED: a longer
  sweep on demand.
"""
import os

import numpy as np
import pytest

from helpers import CODES, Oracle, random_frames

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from convolutionalencdec_amd import ConvCode, ViterbiDecoder, native  # noqa: E402

THREADS = min(16, os.cpu_count() or 1)
FIX_ALL = 1 << 15    # VTB_DEBUG: fix-up on every split frame
FIX_NEVER = 1 << 16  # VTB_DEBUG: fix-up checkpoints never match (slow path after kFix chunks)
SEG_OFF = 1 << 10    # VTB_DEBUG: no single-frame SEG kernel (the frame kernel decodes)
SIGMA = {0.0: 0.3, 0.03: 0.56, 0.07: 0.7, 0.5: 4.0}


@pytest.fixture(scope="module")
def orc():
    return Oracle()


@pytest.fixture(scope="module", autouse=True)
def gpu_present():
    if not torch.cuda.is_available() or native.lib().vtb_device_count() < 1:
        pytest.fail("no gfx950 GPU visible to the C ABI (GPU tests must not silently pass)")


def _frames(orc, L, F, soft, noise, seed):
    if soft:
        unc, x = random_frames(orc, 7, L, F, 0.0, seed, soft=True, sigma=SIGMA[noise])
    else:
        unc, x = random_frames(orc, 7, L, F, noise, seed)
    return unc, np.ascontiguousarray(x).reshape(F, -1)


def _bad_bits(got, want, L):
    g = np.unpackbits(got, axis=1)[:, :L]
    w = np.unpackbits(want, axis=1)[:, :L]
    return [(int(f), np.flatnonzero(g[f] != w[f])[:8].tolist()) for f in np.flatnonzero((g != w).any(axis=1))]


# ---------------------------------------------------------------- case 1366 (round 3) --

L1366 = 2966


@pytest.fixture(scope="module")
def case1366(orc):
    # tests/test_gpu_fuzz.py _frame_cases(seed 1018): case 1366 = K7 L2966 soft p0.5, frames
    # from random_frames(..., 5000 + 1366)
    unc, x = _frames(orc, L1366, 3, True, 0.5, 5000 + 1366)
    want = orc.decode(7, CODES[7], x, L1366, soft=True, threads=THREADS)
    return x, want


@pytest.mark.parametrize("dbg", [0, FIX_ALL, FIX_ALL | FIX_NEVER], ids=["default", "fix_all", "fix_never"])
def test_case_1366_batch(case1366, dbg, monkeypatch):
    """vtb_decode_device on the three frames: the non-persistent split kernel (k7_lds_split)."""
    x, want = case1366
    monkeypatch.delenv("VTB_KERNEL", raising=False)
    monkeypatch.setenv("VTB_DEBUG", str(dbg))
    d = ViterbiDecoder(ConvCode(7, CODES[7]), frame_bits=L1366, soft=True)
    got = d.decode_device(torch.from_numpy(x).cuda()).cpu().numpy()
    assert native.last_kernel() == "k7_lds_split"
    assert (got == want).all(), _bad_bits(got, want, L1366)


@pytest.mark.parametrize("dbg", [0, SEG_OFF, SEG_OFF | FIX_ALL], ids=["default", "seg_off", "seg_off_fix_all"])
def test_case_1366_single_frame(case1366, dbg, monkeypatch):
    """vtb_decode_frame_sync frame by frame (SEG kernel, and on a miss the split frame kernel)."""
    x, want = case1366
    monkeypatch.delenv("VTB_KERNEL", raising=False)
    monkeypatch.setenv("VTB_DEBUG", str(dbg))
    d = ViterbiDecoder(ConvCode(7, CODES[7]), frame_bits=L1366, soft=True)
    got = np.stack([d.decode_frame(r) for r in x])
    assert (got == want).all(), _bad_bits(got, want, L1366)


def test_case_1366_frame1_every_entry(case1366, monkeypatch):
    """Frame 1 alone (the frame that failed) and the batch in reverse order."""
    x, want = case1366
    monkeypatch.delenv("VTB_KERNEL", raising=False)
    monkeypatch.delenv("VTB_DEBUG", raising=False)
    d = ViterbiDecoder(ConvCode(7, CODES[7]), frame_bits=L1366, soft=True)
    got1 = d.decode_device(torch.from_numpy(x[1:2].copy()).cuda()).cpu().numpy()
    assert (got1 == want[1:2]).all(), _bad_bits(got1, want[1:2], L1366)
    rev = d.decode_device(torch.from_numpy(x[::-1].copy()).cuda()).cpu().numpy()
    assert (rev == want[::-1]).all(), _bad_bits(rev, want[::-1], L1366)


# ---------------------------------------------------------------- fix-up family --

FIXUP_N = int(os.environ.get("VTB_FIXUP_N", "0"))
FIXUP_SEED = int(os.environ.get("VTB_FIXUP_SEED", "0"))

# Upper frame lengths per kernel: k7_lds_split needs split_t1(T) <= 32 blocks of 48 steps
# (T <= 2,976); k7_split_loop needs the half's survivor words to leave 8 waves per CU
# (vtb_k7_lds.hip split_loop_params: T up to about 2,060, C3's 2,054 at warm-up 48).
L_MAX = {"split": 2966, "loop": 2050}


def _fixup_cases(n=FIXUP_N or 240, seed=FIXUP_SEED or 20261101):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        kern = "loop" if i % 2 else "split"
        # T = L + 6 over every residue mod 96 (the split point and the fix-up's chunk grid
        # depend on T mod 48 and mod 96), lengths up to the kernel's limit
        r = (37 * i) % 96
        kmax = (L_MAX[kern] + 6 - r) // 96
        T = 96 * int(rng.integers(3, kmax + 1)) + r
        L = T - 6
        if kern == "split":
            # frames the CUs hold at one frame per wave (k7_launch: split below that count)
            F = int(rng.choice([1, 2, 3, 65, 2048]))
            if F == 2048 and L > 1000:
                F = 65
        else:
            F = int(rng.choice([1, 2, 3, 65, 2048, 8192]))
        soft = bool(rng.integers(0, 2))
        noise = float(rng.choice([0.0, 0.03, 0.07, 0.5]))
        dbg = int(rng.choice([FIX_ALL, FIX_ALL, FIX_ALL | FIX_NEVER, 0]))
        out.append((i, kern, L, F, soft, noise, dbg))
    # the persistent C3 shape (65,536 x 2,048 soft at the bench's -5 dB noise, and hard)
    out.append((n, "loop", 2048, 65536, True, 0.03, FIX_ALL))
    out.append((n + 1, "loop", 2048, 65536, False, 0.07, FIX_ALL | FIX_NEVER))
    return out


def _fid(c):
    i, kern, L, F, soft, noise, dbg = c
    mode = {0: "plain", FIX_ALL: "fixall", FIX_ALL | FIX_NEVER: "fixnever"}[dbg]
    return f"{i}-{kern}-L{L}-T{L + 6}m96_{(L + 6) % 96}-F{F}-{'soft' if soft else 'hard'}-p{noise}-{mode}"


@pytest.mark.parametrize("case", _fixup_cases(), ids=_fid)
def test_fixup_family_vs_oracle(orc, case, monkeypatch):
    i, kern, L, F, soft, noise, dbg = case
    unc, x = _frames(orc, L, F, soft, noise, 9000 + i)
    want = orc.decode(7, CODES[7], x, L, soft=soft, threads=THREADS)
    monkeypatch.setenv("VTB_DEBUG", str(dbg))
    if kern == "loop":
        monkeypatch.setenv("VTB_KERNEL", "k7s")
    else:
        monkeypatch.delenv("VTB_KERNEL", raising=False)
    d = ViterbiDecoder(ConvCode(7, CODES[7]), frame_bits=L, soft=soft)
    got = d.decode_device(torch.from_numpy(x).cuda()).cpu().numpy()
    name = native.last_kernel()
    assert name == ("k7_split_loop" if kern == "loop" else "k7_lds_split"), name
    bad = _bad_bits(got, want, L)
    assert not bad, (case, len(bad), bad[:4])
    if noise == 0.0:
        assert (got == unc).all()
