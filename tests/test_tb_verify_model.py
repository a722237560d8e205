"""CPU: a model of the block-parallel traceback's verification loop and its completeness guard
(DESIGN.md 4.0 "Traceback rule", 4.2b), checked against the round cap of every loop in the kernels.

Each lane walks one block of a chain from an unverified start; a block is proven when it entered
on its successor's exit and every later block is proven (the chain's last block is known).  A
round checks every block, then re-walks each failed block whose successors are all proven from
its successor's exit, so the proven suffix grows by at least one block per round: a chain of n
blocks needs at most n - 1 re-walk rounds.  Round 3 capped the split pass's loop at 33 rounds
although its chain has up to 63 blocks, and shipped wrong bits (fuzz case 1366).  Since round 5
every loop is

    for (round = 0;; round++) { check; if all proven: break; if round == cap: guard; re-walk }

and the guard sends a chain still unproven after `cap` re-walk rounds to the exact slow path
(tests/test_gpu_tb_guard.py).  This file models that loop and checks each kernel's cap against
the longest chain its geometry allows.
"""
import os
import re

import numpy as np
import pytest

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "convolutionalencdec_amd", "csrc")


def verify(entry_top, walk, start_exit, cap, force=False):
    """The kernel loop over one chain (block i's successor is i + 1; the last block is known).
    entry_top[i]: the location block i's first walk reached at its top; walk(i, loc): block i's
    exit walked from loc; start_exit[i]: its exit from the first walk.  force: VTB_DEBUG bit 17
    (no check counts, cap 0).  Returns (re-walk rounds used, proven, guard fired)."""
    n = len(entry_top)
    fin = list(start_exit)
    fixed = [False] * (n - 1) + [True]
    if force:
        cap = 0
    rnd = 0
    while True:
        ok = [fixed[i] or (entry_top[i] == fin[i + 1] and not force) for i in range(n - 1)] + [True]
        bad = [not o for o in ok]
        if not any(bad):
            return rnd, True, False
        if rnd == cap:
            return rnd, False, True
        succ_proven = [not any(bad[i + 1:]) for i in range(n)]
        new_fin = list(fin)
        for i in range(n - 1):  # the lanes act at once, on this round's state
            if bad[i] and succ_proven[i]:
                new_fin[i] = walk(i, fin[i + 1])
                fixed[i] = True
        fin = new_fin
        rnd += 1


def adversarial_chain(n, seed=0):
    """Every block's first walk is wrong (its top location is never its successor's exit)."""
    rng = np.random.default_rng(seed)
    table = rng.integers(0, 64, (n, 64))
    start_exit = [int(x) for x in rng.integers(0, 64, n)]
    return [64] * n, (lambda i, loc: int(table[i, loc])), start_exit


@pytest.mark.parametrize("n", [2, 32, 33, 62, 63, 64])
def test_rewalk_rounds_needed(n):
    top, walk, ex = adversarial_chain(n)
    assert verify(top, walk, ex, 10 * n) == (n - 1, True, False)
    assert verify(top, walk, ex, n - 1)[1]            # a cap of n - 1 suffices
    if n > 2:
        assert verify(top, walk, ex, n - 2)[2]        # one less fires the guard


def test_round3_split_bound_fires_guard():
    """The round-3 cap (33) on a 62-block split chain now fires the guard instead of shipping
    the first blocks unverified; the shipped cap (65) proves it."""
    top, walk, ex = adversarial_chain(62, seed=1)
    assert verify(top, walk, ex, 33) == (33, False, True)
    assert verify(top, walk, ex, 65)[:2] == (61, True)


def test_forced_guard_fires_on_every_walked_chain():
    """VTB_DEBUG bit 17: every chain with a block not known from the frame end takes the guard,
    even one whose first walks all verified; a chain of known blocks only does not."""
    for n in (2, 32, 64):
        top, walk, ex = adversarial_chain(n, seed=n)
        assert verify(top, walk, ex, 65, force=True) == (0, False, True)
    top, walk, ex = adversarial_chain(8, seed=3)
    good = [walk(i + 1, 0) if i < 7 else 0 for i in range(8)], walk, [walk(i, 0) for i in range(8)]
    assert verify(*good, 65)[:2] == (0, True)
    assert verify(*good, 65, force=True) == (0, False, True)
    assert verify([0], walk, [0], 65, force=True) == (0, True, False)


def _caps(fname):
    src = open(os.path.join(CSRC, fname)).read()
    caps = re.findall(r"const int rounds = tbforce \? 0 : ([^;]+);", src)
    # (tbforce: VTB_DEBUG bit 17 read in the kernel, or passed in by it -- traceback_chains)
    assert (len(re.findall(r"const bool tbforce = \((?:table\.|a\.)?dbg & kDbgTbCap\) != 0;", src))
            + len(re.findall(r"\bbool tbforce,", src))) == len(caps)
    # bit 17 makes no check pass: the entry location poisoned (K=7 / K=9) or the check masked
    forced = (len(re.findall(r"if \(tbforce\) loc_top = ~0u;", src))
              + len(re.findall(r"const bool okb? = fixed \|\| \(\w+ == \w+ && !tbforce\);", src)))
    assert forced == len(caps), (fname, forced, len(caps))
    loops = len(re.findall(r"for \(int round = 0;; round\+\+\)", src))
    assert len(caps) == loops, (fname, caps, loops)
    assert not re.search(r"for \(int round = 0; round <", src), f"{fname}: an unguarded verification loop"
    assert len(re.findall(r"if \(round == rounds\)", src)) == loops, fname
    return caps


def test_every_loop_cap_covers_its_chain():
    """Each loop's cap against the longest chain its geometry allows (n - 1 re-walks)."""
    k7 = _caps("vtb_k7_lds.hip")
    # k7_pair: unsplit frames chain their 32 blocks; the split pass chains frame A's nA <= 32
    # blocks (t1 <= 32 * 48, split_loop_params / k7_launch) and frame B's lanes kB0..63 with
    # kB0 = 32 + warm / 48 >= 33 (warm >= 48): nA + 64 - kB0 <= 63 blocks.
    # (source order: stream_traceback, k7_pair, k7_seg_kernel)
    assert k7 == ["33", "(SPLIT && sp) ? 65 : 33", "65"]
    assert 65 >= 63 - 1 and 33 >= 32 - 1
    src = open(os.path.join(CSRC, "vtb_k7_lds.hip")).read()
    assert "const int kB0 = 32 + warm / kChunk;" in src
    assert "if (t1 > 32 * kChunk) return false;" in src and "warm >= kChunk" in src
    # stream_traceback: 32 blocks per frame; k7_seg_kernel: one chain over the 64 lanes
    k9 = _caps("vtb_k9.hip")
    # stream (32 blocks), frame pair (32 per frame), SEG (64), one frame per wave (k9s: 64 blocks)
    assert k9 == ["33", "33", "65", "65"]
    src9 = open(os.path.join(CSRC, "vtb_k9.hip")).read()
    assert "const int per = (Tq + 31) / 32;" in src9 and "const int per = (Tq + 63) / 64;" in src9
    assert _caps("vtb_genk.hip") == ["65"]  # one chain over the 64 lanes
    # generic batch, single-frame and stream kernels share traceback_span: GC lanes (blocks) per
    # chain, GC = G (lds_path_kernel, gen_stream_kernel: one stream's lanes) or 64 (gen_seg_kernel)
    assert _caps("vtb_gen_trellis.h") == ["GC + 1"]
    assert _caps("vtb_lds_path.hip") == []
    src = open(os.path.join(CSRC, "vtb_lds_path.hip")).read()
    assert src.count("traceback_chains<S, R>(T, L, G,") == 1 and src.count("traceback_chains<S, R>(T, L, 64,") == 1
    assert _caps("vtb_stream_gen.hip") == []
    src = open(os.path.join(CSRC, "vtb_stream_gen.hip")).read()
    assert src.count("traceback_span<S, R>(e0, emits ? hi : e0, emit_end, rotr_s<S>(kloc, hi % S), G,") == 1


@pytest.mark.parametrize("fname", ["vtb_k7_lds.hip", "vtb_k9.hip", "vtb_genk.hip", "vtb_gen_trellis.h"])
def test_every_guard_has_a_slow_path(fname):
    """After each loop an unproven chain reaches an exact slow path, and the testing counter
    notes it (note_guard)."""
    src = open(os.path.join(CSRC, fname)).read()
    loops = len(re.findall(r"for \(int round = 0;; round\+\+\)", src))
    assert len(re.findall(r"note_guard\(", src)) >= loops
