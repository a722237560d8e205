"""CPU: worst-case u16 headroom of the K=7 kernel's packed metrics (vtb_k7_lds.hip; DESIGN.md 3,
4.1 and 5), for every input.

The ACS keeps [frame A, frame B] metrics as u16 halves of one register, each SC·m + h (SC = 4
for 8-bit soft input with 2 history bits, 256 for hard input with 8).  A carry out of a half
would corrupt the other frame, and random frames never come near the worst case, so the
bounds are checked here on the arithmetic itself, from the constants in the kernel source:

* renormalisation: location 0's metric is read at step RN - 2 of each period (soft; hard: step
  40 of the 48-step chunk) and subtracted, plus the bias B, at step RN - 1 (hard: 47);
* spread: for t >= 6 every state is within (K - 1)·n·Q of every other (reference
  viterbiDecoderButterflyk1.c:159-183 relies on the same bound for its uint8 renorm);
* padding rows (steps past T) make every location keep its own predecessor by adding
  W = SC·INIT to the partner candidate, INIT = (K - 1)·n·Q + 1 (vtb_k7_lds.hip stage_write).

Round 4 found that the round-2 argument for a 16-step soft period omitted the padding rows
(PERF_LOG.md 5); these tests pin the shipped period and show why 16 does not fit.
"""
import os
import re

import pytest

SRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   "convolutionalencdec_amd", "csrc", "vtb_k7_lds.hip")
U16 = 1 << 16


def shipped_period():
    m = re.search(r"constexpr int kRenormSoft = (\d+);", open(SRC).read())
    assert m, "soft renormalisation period not found"
    return int(m.group(1))


def worst_candidate(soft, nb, period=None):
    """Largest u16 value a candidate (own or partner, padding rows included) can take."""
    q = 255 if soft else 1
    sc = 4 if soft else 256
    hist = sc - 1                       # history bits below the metric
    emax = nb * q                       # largest branch metric of one step
    spread = 6 * nb * q                 # (K - 1)·n·Q, K = 7
    init = spread + 1                   # start metric of states != 0, and the padding W / SC
    bias = 3060 if soft else 6 * nb     # H::BIAS / SC
    if soft:
        read, apply, between = period - 2, period - 1, period
    else:
        read, apply, between = 40, 47, 48
    # after an apply: m - m_loc0(read) + B, the reference taken (apply - read + 1) steps earlier
    m_after = bias + spread + (apply - read + 1) * emax
    # the last candidates before the next apply are formed from metrics grown for between - 1 steps
    m_top = m_after + (between - 1) * emax
    # before the first renormalisation: the start metrics plus growth
    m_first = bias + init + (apply + 1) * emax
    m = max(m_top, m_first)
    tie = sc // 2                       # the tie bit at the top history position
    own = sc * (m + emax) + hist + tie
    partner_padding = sc * m + hist + sc * init + tie
    return max(own, partner_padding), m


@pytest.mark.parametrize("soft,nb", [(True, 2), (False, 2), (False, 3)],
                         ids=["soft", "hard", "hard-rate1/3"])
def test_shipped_metrics_fit_u16(soft, nb):
    worst, m = worst_candidate(soft, nb, shipped_period())
    assert worst < U16, (worst, m)
    if not soft:
        assert m < 256  # hard input keeps 256m + h: the metric itself must fit 8 bits


def test_soft_period_16_overflows_padding():
    """The rejected 16-step soft period: a padding step's partner candidate can carry out."""
    worst, _ = worst_candidate(True, 2, 16)
    assert worst >= U16


def test_shipped_soft_period_is_12():
    assert shipped_period() == 12


K9_SRC = os.path.join(os.path.dirname(SRC), "vtb_k9.hip")


def worst_candidate_k9(soft, nb):
    """The same worst case for the K=9 kernel (vtb_k9.hip): bias B = SC·8·n·Q (8 = K - 1), a
    12-step soft period (steps 10 / 11) or one renormalisation per 48-step chunk (hard, steps
    40 / 47); soft padding steps run on clamped input (their survivor bits are overwritten
    after the ACS), hard padding rows add W = SC·(8·n·Q + 1)."""
    q = 255 if soft else 1
    sc = 4 if soft else 256
    emax, spread = nb * q, 8 * nb * q
    bias = spread
    read, apply, between = (10, 11, 12) if soft else (40, 47, 48)
    m_after = bias + spread + (apply - read + 1) * emax
    m = max(m_after + (between - 1) * emax, bias + q + (apply + 1) * emax)  # start value (uint8)(257)·Q = Q
    tie = sc // 2
    own = sc * (m + emax) + (sc - 1) + tie
    pad = 0 if soft else sc * m + (sc - 1) + sc * (spread + 1) + tie
    return max(own, pad), m


def test_k9_constants_match_model():
    src = open(K9_SRC).read()
    assert "constexpr uint32_t B4 = H::SC * 8 * NB * Q;" in src
    assert "PADW = H::SC * ((SOFT ? 2 : 8 * NB) * Q + 1) * kR1;" in src
    assert re.search(r"RN_READ = SOFT \? \(I % 12\) == 10 : I == 40;", src)
    assert re.search(r"RN_APPLY = SOFT \? \(I % 12\) == 11 : I == 47;", src)


@pytest.mark.parametrize("soft,nb", [(True, 2), (False, 2), (False, 3)],
                         ids=["soft", "hard", "hard-rate1/3"])
def test_k9_metrics_fit_u16(soft, nb):
    worst, m = worst_candidate_k9(soft, nb)
    assert worst < U16, (worst, m)
    if not soft:
        assert m < 256


def test_k7_constants_match_model():
    src = open(SRC).read()
    assert "constexpr uint32_t INIT = 6 * NB * Q + 1;" in src
    assert "static constexpr uint32_t BIAS = SC * (SOFT ? 3060 : 6 * NB);" in src
    assert "constexpr uint32_t PADW = H::SC * INIT * kR1;" in src
    assert "#define VTB_RENORM_READ(I) (SOFT ? ((I) % kRenormSoft) == kRenormSoft - 2 : (I) == 40)" in src
    assert "#define VTB_RENORM_APPLY(I) (SOFT ? ((I) % kRenormSoft) == kRenormSoft - 1 : (I) == 47)" in src
