"""CPU: a model of the block-parallel traceback's verification loop (vtb_k7_lds.hip, k7_pair
"traceback: verified block-parallel chains") and its round bound.

Each lane walks one block of a chain from an unverified start; a block is proven when it
entered on its successor's exit and every later block is proven.  Every round re-walks the
failed blocks whose successors are all proven, so at least the last unproven block becomes
proven per round.  A chain of n blocks therefore needs at most n rounds plus the round that
sees no failure.  Round 3 capped the loop at 33 rounds for every chain, but the split pass
chains frame A's nA <= 32 blocks and frame B's blocks 2..31 (up to 62): with blocks that keep
failing (pure-noise frames whose paths do not merge within the walk warm-up) the first
blocks of frame A left the loop unverified (fuzz case 1366).  The kernel now allows 65
rounds for split chains (the `rounds` bound); this model pins that arithmetic.
"""
import os
import re

import numpy as np
import pytest

KERNEL = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                      "convolutionalencdec_amd", "csrc", "vtb_k7_lds.hip")


def verify_rounds(entry_top, walk, start_exit, max_rounds):
    """Run the kernel's verification rounds over one chain (block i's successor is i + 1; the
    last block is known).  entry_top[i]: the location block i's first walk reached at its top;
    walk(i, loc): block i's exit when walked from loc; start_exit[i]: its exit from the first
    walk.  Returns (rounds used, all proven)."""
    n = len(entry_top)
    fin = list(start_exit)
    fixed = [False] * (n - 1) + [True]
    for rnd in range(max_rounds):
        ok = [fixed[i] or (entry_top[i] == fin[i + 1]) for i in range(n - 1)] + [True]
        bad = [not o for o in ok]
        if not any(bad):
            return rnd + 1, True
        # the kernel's lanes act at once, on this round's state
        succ_proven = [not any(bad[i + 1:]) for i in range(n)]
        new_fin = list(fin)
        for i in range(n - 1):
            if bad[i] and succ_proven[i]:
                new_fin[i] = walk(i, fin[i + 1])
                fixed[i] = True
        fin = new_fin
    ok = [fixed[i] or (entry_top[i] == fin[i + 1]) for i in range(n - 1)] + [True]
    return max_rounds, all(ok)


def adversarial_chain(n, seed=0):
    """Every block's first walk is wrong (its top location is never its successor's exit)."""
    rng = np.random.default_rng(seed)
    exits = rng.integers(0, 64, n)
    table = rng.integers(0, 64, (n, 64))
    start_exit = [int(x) for x in exits]
    # entry_top never matches any exit a successor can produce: use 64 (no such location)
    entry_top = [64] * n
    return entry_top, (lambda i, loc: int(table[i, loc])), start_exit


@pytest.mark.parametrize("n", [32, 33, 62, 63])
def test_rounds_needed_is_chain_length(n):
    top, walk, ex = adversarial_chain(n)
    used, proven = verify_rounds(top, walk, ex, 10 * n)
    assert proven and used == n  # n - 1 unproven blocks, one per round, plus the clean round


def test_split_chain_exceeds_round3_bound():
    """62-block split chains: 33 rounds leave the first blocks unproven; 65 do not."""
    top, walk, ex = adversarial_chain(62, seed=1)
    assert verify_rounds(top, walk, ex, 33) == (33, False)
    used, proven = verify_rounds(top, walk, ex, 65)
    assert proven and used <= 65


def test_unsplit_chain_fits_33():
    top, walk, ex = adversarial_chain(32, seed=2)
    assert verify_rounds(top, walk, ex, 33)[1]


def test_kernel_round_bounds():
    """The shipped kernel allows 65 rounds on split chains (up to 62 blocks: frame A's nA <= 32
    and frame B's blocks kB0..63 with kB0 >= 33) and 33 on unsplit ones (32 blocks)."""
    src = open(KERNEL).read()
    m = re.search(r"const int rounds = \(SPLIT && sp\) \? (\d+) : (\d+);", src)
    assert m, "verification round bound not found in vtb_k7_lds.hip"
    split_rounds, frame_rounds = int(m.group(1)), int(m.group(2))
    longest_split_chain = 32 + (64 - 33)  # nA <= 32 blocks, frame B's lanes kB0 = 32 + warm/48 >= 33 .. 63
    assert split_rounds >= longest_split_chain + 1
    assert frame_rounds >= 32 + 1
