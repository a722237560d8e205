"""CPU model of the K=9 one-frame-per-wave layout (k9s, vtb_k9.hip).

k9s holds one frame's 256 locations as l = 128 h + 64 r + lambda (u16 half h, register r, lane
location lambda) and builds its branch-metric table from the pair kernel's, with the high half of
every column describing location l ^ 128 instead of another frame.  This restates, in Python, what
the kernel does and checks it against the pair kernel's own per-location definitions (the butterfly
of /root/reference/src/viterbiDecoderButterflyk1.c:101-152 as k9_pair lays it out):

* the column a high-half location needs is the low location's column with the label XORed by
  d(ph) (ph >= 1) or R flipped (ph = 0): butterfly labels are linear in the state for every code
  vtb_edge_table accepts, so k9s_dpack never refuses one;
* the staging lane's packed (V, W) values -- input complemented by d(ph) for the high half, tie
  bit moved to the other half at ph = 0 -- equal, half by half, the values each location reads in
  the pair kernel's table, for soft and hard input and for the own-keeping rows;
* the survivor word of (lane, register, half) sits at byte 2 l' (l' = rev8(l)), so a window's two
  decisions are the contiguous address bits the traceback edits.
"""
import os

import numpy as np
import pytest

from helpers import CODES, load_golden

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "convolutionalencdec_amd", "csrc")

K = 9


def rev(x, n):
    return int(format(x, f"0{n}b")[::-1], 2)


def parity(x):
    return bin(x).count("1") & 1


def edge_table(g):
    """vtb_api.hip edge_table (viterbiInitButterflyk1, reference viterbiDecoderButterflyk1.c:8-44)."""
    p0, p1 = rev(g[0], K), rev(g[1], K)
    return [parity((i << 1) & p0) | (parity((i << 1) & p1) << 1) for i in range(1 << (K - 2))]


def lane_of(lam):
    return lam ^ (((lam >> 2) & 1) * 3)


def rotl8(x, r):
    return ((x << r) | (x >> (8 - r))) & 255


def column(symm, l, ph):
    """k9_pair column_offsets / k9s_kernel: (label c of the butterfly's upper state, R = bit p)."""
    p = 7 - ph
    return symm[rotl8(l & ~(1 << p), ph)], (l >> p) & 1


def dpack(symm):
    """k9s_dpack, or None where it refuses the code."""
    out = 0
    for ph in range(1, 8):
        e = 1 << (ph - 1)
        d = symm[e] ^ symm[0]
        if d > 3 or any((symm[s ^ e] ^ symm[s]) != d for s in range(128)):
            return None
        out |= d << (2 * ph)
    return out


def test_restated_edge_table_is_the_references():
    """The restatement above against the reference's own table (golden vector from the reference
    build, tests/golden/edge_tables.npz)."""
    assert edge_table(CODES[K]) == [int(x) for x in load_golden("edge_tables.npz")["k9"]]


def test_model_follows_the_kernel_source():
    """The lines of k9_single / k9s_dpack this model restates."""
    src = open(os.path.join(CSRC, "vtb_k9.hip")).read()
    for line in ("const uint32_t xmask = SOFT ? ((d & 1u) ? 0xFFu : 0u) | ((d & 2u) ? 0xFF00u : 0u) : d;",
                 "const uint32_t tieE = sph == 0 ? tie16 << 16 : 0u, tieT = sph == 0 ? tie16 : tie16 * kR1;",
                 "const uint32_t rb = ra ^ xmask;",
                 "const int d = a.symm[e] ^ a.symm[0];",
                 "col[k * kCol] = make_uint2(tieE, PADW + tieT);",
                 "col[(4 + k) * kCol] = make_uint2(tieT, PADW + tieE);",
                 "const uint32_t wlane = 8u * rev6(lam);",
                 "const int pos = ((todd - 1) & 7) + 1;"):
        assert line in src, line


def valid_codes(n, seed):
    rng = np.random.default_rng(seed)
    codes = [CODES[K]]
    while len(codes) < n:
        g = tuple(int(x) | 1 | (1 << (K - 1)) for x in rng.integers(0, 1 << K, 2))
        codes.append(g)
    return codes


@pytest.mark.parametrize("g", valid_codes(24, 9), ids=lambda g: f"{g[0]:o}_{g[1]:o}")
def test_high_half_column_is_the_partner_locations(g):
    symm = edge_table(g)
    dp = dpack(symm)
    assert dp is not None, "labels are linear in the state: k9s_dpack accepts every valid code"
    for ph in range(8):
        d = (dp >> (2 * ph)) & 3
        for l0 in range(128):
            c, R = column(symm, l0, ph)
            want = column(symm, l0 ^ 128, ph)
            got = (c, 1 - R) if ph == 0 else (c ^ d, R)
            assert got == want, (ph, l0)


def staged_columns(raw, srow, soft, xmask_of, tie_split):
    """The packed (V, W) of the 8 columns as k9s stage_compute / stage_write build row srow."""
    HB = 2 if soft else 8
    SC, Q = 1 << HB, 255 if soft else 1
    QQ = SC * Q

    def e_of(r):
        if soft:
            q0, q1 = (r & 0xFF) << HB, ((r >> 8) & 0xFF) << HB
        else:
            q0, q1 = (r & 1) << HB, ((r >> 1) & 1) << HB
        e0, e1 = q0 + q1, QQ + q1 - q0
        return [e0, e1, 2 * QQ - e1, 2 * QQ - e0]

    ph = srow & 7
    lo, hi = e_of(raw), e_of(raw ^ xmask_of(ph))
    tie = 1 << (srow & (HB - 1))
    tieE, tieT = tie_split(ph, tie)  # (lo, hi) pairs added to e / et
    e = [(lo[k] + tieE[0], hi[k] + tieE[1]) for k in range(4)]
    et = [(lo[k] + tieT[0], hi[k] + tieT[1]) for k in range(4)]
    cols = {}
    for c in range(4):
        cols[(c, 0)] = (e[c], et[3 - c])
        cols[(c, 1)] = (et[c], e[3 - c])
    return cols, e_of(raw), tie


@pytest.mark.parametrize("soft", [True, False], ids=["soft", "hard"])
@pytest.mark.parametrize("g", valid_codes(6, 11), ids=lambda g: f"{g[0]:o}_{g[1]:o}")
def test_staged_values_equal_each_locations_own(soft, g):
    symm = edge_table(g)
    dp = dpack(symm)

    def xmask_of(ph):  # k9_single: the high half's coded bits complemented by d(ph)
        d = (dp >> (2 * ph)) & 3
        return ((0xFF if d & 1 else 0) | (0xFF00 if d & 2 else 0)) if soft else d

    def tie_split(ph, tie):  # tieE / tieT: at ph = 0 the high half takes the other R's tie
        return ((0, tie), (tie, 0)) if ph == 0 else ((0, 0), (tie, tie))

    rng = np.random.default_rng(5)
    for srow in range(48):
        ph = srow & 7
        for raw in rng.integers(0, 1 << 16 if soft else 4, 12):
            raw = int(raw)
            cols, e_direct, tie = staged_columns(raw, srow, soft, xmask_of, tie_split)
            for l0 in range(128):
                V, W = cols[column(symm, l0, ph)]
                for half, l in ((0, l0), (1, l0 ^ 128)):
                    c, R = column(symm, l, ph)
                    want = (e_direct[c] + R * tie, e_direct[3 - c] + (1 - R) * tie)
                    assert (V[half], W[half]) == want, (srow, raw, l0, half)


@pytest.mark.parametrize("soft", [True, False], ids=["soft", "hard"])
def test_own_keeping_rows(soft):
    """The start row of odd T (and hard input's padding rows): every location keeps its own
    predecessor, V = R tie, W = PADW + (1 - R) tie, for both halves' locations."""
    symm = edge_table(CODES[K])
    HB = 2 if soft else 8
    PADW = (1 << HB) * ((2 if soft else 16) * (255 if soft else 1) + 1)
    for srow in range(48):
        ph = srow & 7
        tie = 1 << (srow & (HB - 1))
        tieE, tieT = ((0, tie), (tie, 0)) if ph == 0 else ((0, 0), (tie, tie))
        col = {0: (tieE, (PADW + tieT[0], PADW + tieT[1])), 1: (tieT, (PADW + tieE[0], PADW + tieE[1]))}
        for l0 in range(128):
            _, R0 = column(symm, l0, ph)
            V, W = col[R0]
            for half, l in ((0, l0), (1, l0 ^ 128)):
                _, R = column(symm, l, ph)
                assert (V[half], W[half]) == (R * tie, PADW + (1 - R) * tie), (srow, l0, half)


def test_survivor_word_address_is_2_lprime():
    """k9_single: the word of (lane, register r) at 8 rev6(lambda) + 4 r, the location's u16 at
    + 2 h; the traceback reads 2 l' (tbs_body) and edits l' bits e, e + 1 at address bits e + 1."""
    for lane in range(64):
        lam = lane_of(lane)
        assert lane_of(lam) == lane  # the lane involution
        for r in range(2):
            for h in range(2):
                l = 128 * h + 64 * r + lam
                assert 8 * rev(lam, 6) + 4 * r + 2 * h == 2 * rev(l, 8), (lane, r, h)
    for todd in range(1, 48, 2):  # (todd - 1) & 7 is even: the window's two bits fit in l' bits 0..7
        e = (todd - 1) & 7
        assert e % 2 == 0 and e + 1 <= 7 and ((todd - 1) & 7) + 1 == e + 1
