"""CPU: a numpy model of the generic register-resident trellis (csrc/vtb_gen_trellis.h, DESIGN.md
§4.4) and of the generic single-frame segments (gen_seg_kernel), decoded against
the oracle (itself pinned to the reference build, test_oracle.py).

The model restates the kernels' arithmetic location by location: location l holds state
rotl_S(l, t mod S) before step t; its partner is l ^ (1 << (S-1-phase)); the own candidate is
m[l] + mu and the partner's m[partner] - mu, with mu = sig . rx + kap from the code's edge label
of butterfly j = rotl_S(l, phase) & (N/2 - 1); the decision is ((a - b) ^ up) > up with up = -1
where the location holds the upper predecessor; the new metric min(a, b).  Decision words are
laid out as the kernels lay them out (bit lane_of(l mod 64) of word l >> 6) and the traceback
walks locations (one bit replaced per step).  The segment model uses the kernel's own geometry
rule (gen_seg_geometry) and boundary test."""
import numpy as np
import pytest

from helpers import Oracle, random_frames

CODES = {3: (0o7, 0o5), 4: (0o15, 0o17), 5: (0o23, 0o35), 6: (0o53, 0o75), 7: (0o133, 0o171),
         8: (0o247, 0o371), 9: (0o561, 0o753)}


@pytest.fixture(scope="module")
def orc():
    return Oracle()


def rev(x, n):
    return int(format(x, f"0{n}b")[::-1], 2)


def edge_labels(K, g):
    """vtb_api.hip edge_table: label of the edge j -> 2j (input 0) for the butterflies j."""
    p0, p1 = rev(g[0], K), rev(g[1], K)
    par = lambda v: bin(v).count("1") & 1  # noqa: E731
    return np.array([par((i << 1) & p0) | (par((i << 1) & p1) << 1) for i in range(1 << (K - 2))])


def lane_of(S, l):
    return l ^ (((l >> 2) & 1) * 3) if S >= 3 else l


def rotl(S, x, k):
    N = 1 << S
    return ((x << k) | (x >> (S - k))) & (N - 1)


class Trellis:
    """The kernels' per-location constants for one code (hard: Q = 1, soft: Q = 255)."""

    def __init__(self, K, g, soft):
        self.S = S = K - 1
        self.N = N = 1 << S
        self.Q = Q = 255 if soft else 1
        self.soft = soft
        symm = edge_labels(K, g)
        loc = np.arange(N)
        self.sig0 = np.zeros((S, N), np.int64)
        self.sig1 = np.zeros((S, N), np.int64)
        self.kap = np.zeros((S, N), np.int64)
        self.up = np.zeros((S, N), np.int64)
        self.partner = np.zeros((S, N), np.int64)
        for ph in range(S):
            j = rotl(S, loc, ph) & (N // 2 - 1)
            c = symm[j]
            self.sig0[ph] = np.where(c & 1, -1, 1)
            self.sig1[ph] = np.where(c & 2, -1, 1)
            self.kap[ph] = ((c & 1) + ((c >> 1) & 1) - 1) * Q
            P = S - 1 - ph
            self.up[ph] = -((loc >> P) & 1)
            self.partner[ph] = loc ^ (1 << P)
        self.INIT = ((N + 1) & 0xFF) * Q
        # decision-word bit of each location: word l >> 6, bit lane_of(l mod 64) (G = min(N, 64))
        G = min(N, 64)
        self.word = loc >> 6
        self.bit = np.array([lane_of(S, int(l) % G) for l in loc])

    def rx(self, x, t):
        if self.soft:
            return int(x[2 * t]), int(x[2 * t + 1])
        c = int(x[t])
        return c & 1, (c >> 1) & 1

    def step(self, m, x, t, t_in=None):
        """One step at global step t (phase t mod S) on the received pair of step t_in (default
        t): the new metrics and the decision bits by location."""
        ph = t % self.S
        q0, q1 = self.rx(x, t if t_in is None else t_in)
        mu = self.sig0[ph] * q0 + self.sig1[ph] * q1 + self.kap[ph]
        a = m + mu
        b = m[self.partner[ph]] - mu
        up = self.up[ph]
        dec = ((a - b) ^ up) > up
        return np.minimum(a, b), dec

    def words(self, dec):
        """The R 64-bit decision words of one step, as the kernels store them."""
        R = max(self.N // 64, 1)
        w = [0] * R
        for l in np.nonzero(dec)[0]:
            w[self.word[l]] |= 1 << int(self.bit[l])
        return w

    def walk_bit(self, words, loc):
        G = min(self.N, 64)
        return (words[loc >> 6] >> lane_of(self.S, loc & (G - 1))) & 1


def traceback(tr, rows, T, L):
    """Location walk from state 0 after step T - 1 (the kernels' walk): bits of steps < L."""
    S = tr.S
    loc, bits = 0, np.zeros(T, np.uint8)
    for t in range(T - 1, -1, -1):
        k = (t + 1) % S
        b = 0 if k == 0 else S - k
        bits[t] = (loc >> b) & 1
        x = tr.walk_bit(rows[t], loc)
        loc = (loc & ~(1 << b)) | (x << b)
    return np.packbits(bits[:L])


def decode_model(tr, x, L):
    T = L + tr.S
    m = np.full(tr.N, tr.INIT, np.int64)
    m[0] = 0  # phase 0: location = state
    rows = []
    for t in range(T):
        m, dec = tr.step(m, x, t)
        rows.append(tr.words(dec))
    return traceback(tr, rows, T, L)


@pytest.mark.parametrize("K", [3, 4, 5, 6, 7, 8, 9])
@pytest.mark.parametrize("soft", [False, True])
def test_register_trellis_matches_oracle(orc, K, soft):
    L = 150 + 7 * K
    g = CODES[K]
    if soft:
        unc, rx = random_frames(orc, K, L, 3, 0.0, seed=K, soft=True, sigma=0.7, g=g)
        rx = rx.reshape(3, -1)
    else:
        unc, rx = random_frames(orc, K, L, 3, 0.06, seed=K, g=g)
    want = orc.decode(K, g, rx, L, soft=soft)
    tr = Trellis(K, g, soft)
    for f in range(3):
        assert (decode_model(tr, rx[f], L) == want[f]).all(), (K, soft, f)


def test_lane_map_is_an_involution_and_turns_xor4_into_xor7():
    for S in range(3, 9):
        for l in range(64):
            assert lane_of(S, lane_of(S, l)) == l
            for p, lx in ((0, 1), (1, 2), (2, 7), (3, 8), (4, 16), (5, 32)):
                assert lane_of(S, l ^ (1 << p)) == lane_of(S, l) ^ lx


# ---- single-frame segments (gen_seg_kernel) ----

def body_steps(S):
    return 4 * S if S <= 2 else 2 * S if S <= 4 else S


def gen_seg_geometry(S, T, waves, warm, nwg=1, seg_min=32):
    """vtb_lds_path.hip gen_seg_geometry without the LDS check: (n, warm, G) or None."""
    seg_max = 64 if nwg > 1 or S <= 3 else 32
    F = 64 >> S if S < 6 else 1
    P = body_steps(S)
    warm = (warm + P - 1) // P * P
    G = min(waves * F * nwg, seg_max, (T - warm) // seg_min)
    if G < 2:
        return None
    sstep = (T - warm + G - 1) // G
    sstep = (sstep + P - 1) // P * P
    G = (T - warm + sstep - 1) // sstep
    if G < 2:
        return None
    if nwg > 1 and (G + F - 1) // F <= waves:
        return None  # (one workgroup holds them: the single-workgroup form)
    return sstep + warm, warm, G


def decode_segments(tr, x, L, waves=8, warm=48, nwg=1):
    """The segment decode: None if a boundary did not converge (the kernel's *done = 2)."""
    S, N = tr.S, tr.N
    T = L + S
    geo = gen_seg_geometry(S, T, waves, warm, nwg)
    assert geo is not None
    n, warm, G = geo
    sstep = n - warm
    assert (G - 1) * sstep < T - warm, "a segment starts where it covers nothing"
    assert G * sstep + warm >= T
    rows = [None] * T
    fin, mw = [], []
    for i in range(G):
        g0 = i * sstep
        assert g0 % S == 0  # every slot of a wave shares the phase
        m = np.zeros(N, np.int64)
        if i == 0:
            m[:] = tr.INIT
            m[0] = 0
        for lt in range(n):
            # (steps past the frame: clamped input, their decisions unused)
            m, dec = tr.step(m, x, g0 + lt, min(g0 + lt, T - 1))
            if (i == 0 or lt >= warm) and g0 + lt < T:
                rows[g0 + lt] = tr.words(dec)
            if lt + 1 == warm:
                mw.append(m.copy())
        fin.append(m)
    for i in range(1, G):
        d = fin[i - 1] - mw[i]  # both at phase 0: index = location = state
        if not (d == d[0]).all():
            return None
    assert all(r is not None for r in rows)
    return traceback(tr, rows, T, L)


@pytest.mark.parametrize("K,L,nwg", [(3, 1000, 1), (3, 2048, 1), (4, 1000, 1), (5, 2048, 1), (6, 1000, 1),
                                     (8, 2048, 1), (6, 2048, 4), (8, 2048, 4)])
def test_segments_match_oracle_when_converged(orc, K, L, nwg):
    """(nwg = 4: the shipped form for K = 6, 8 -- up to 64 segments over four workgroups.)"""
    g = CODES[K]
    unc, rx = random_frames(orc, K, L, 2, 0.02, seed=100 + K, g=g)
    want = orc.decode(K, g, rx, L)
    tr = Trellis(K, g, False)
    converged = 0
    for f in range(2):
        got = decode_segments(tr, rx[f], L, nwg=nwg)
        if got is not None:
            converged += 1
            assert (got == want[f]).all(), (K, L, f)
    assert converged >= 1, (K, L)


def test_segment_geometry_never_leaves_a_segment_past_the_frame():
    """The round-6 fix: rounding the segment step up to whole loop bodies can leave the last
    segments nothing to cover; they are dropped (a segment on clamped input need not converge)."""
    for S in range(2, 8):
        if S == 6:
            continue
        for T in range(80, 4200, 37):
            for nwg in (1, 4):
                geo = gen_seg_geometry(S, T, 8, 48, nwg)
                if geo is None:
                    continue
                n, warm, G = geo
                sstep = n - warm
                assert (G - 1) * sstep + warm < T and G * sstep + warm >= T, (S, T, nwg, geo)


def sbfe8(word, offset):
    """v_bfe_i32(word, offset, 8): offset bits 4..0 only, sign-extended byte."""
    v = (word >> (offset & 31)) & 0xFF
    return v - 256 if v >= 128 else v


@pytest.mark.parametrize("K", [3, 4, 5, 6, 7, 8, 9])
def test_hard_metric_table_matches_dot_form(K):
    """Hard input: the kernels read a location's branch metric from a word of four signed bytes
    (vtb_gen_trellis.h setup_coef, rot_step: v_bfe_i32 at offset 8 c, the symbol byte staged as
    hard_offset = (byte & 3) << 3) instead of the v_dot2 form; every symbol byte gives the dot
    form's value of its two low bits (the reference's `coded & 3`)."""
    tr = Trellis(K, CODES[K], False)
    for ph in range(tr.S):
        for l in range(tr.N):
            s0, s1, kap = int(tr.sig0[ph][l]), int(tr.sig1[ph][l]), int(tr.kap[ph][l])
            tab = 0
            for c in range(4):
                tab |= ((s0 * (c & 1) + s1 * (c >> 1) + kap) & 0xFF) << (8 * c)
            for raw in range(256):
                want = s0 * (raw & 1) + s1 * ((raw >> 1) & 1) + kap
                assert sbfe8(tab, (raw & 3) << 3) == want, (K, ph, l, raw)
