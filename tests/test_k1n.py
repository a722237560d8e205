"""k = 1 codes with n != 2: the oracle's restatement of the reference's
k=1 decoder for any n (oracle_k1n_decode, viterbiDecoderButterflyk1.c:82-256 with its
compile-time n) against the reference's own outputs (tests/golden/k1n.npz, made by
make_golden_k1n.py from oracle/_ref/libref_<name>.so), and its relation to exact ML.
CPU only; the GPU path is tests/test_gpu_k1n.py."""
import numpy as np
import pytest

from helpers import CODES, K1N_PARAMS, Oracle, golden_sets, k1n_frames, load_golden


@pytest.fixture(scope="module")
def orc():
    return Oracle()


def k1n_sets(name):
    z = load_golden("k1n.npz")
    keys = sorted({k.rsplit("_", 1)[0] for k in z if k.startswith(name + "_L")})
    assert keys
    for key in keys:
        L = int(key.split("_")[1][1:])
        yield key, L, z[key + "_rx"], z[key + "_decoded"], z[key + "_uncoded"]


@pytest.mark.parametrize("name", sorted(K1N_PARAMS))
def test_oracle_k1n_matches_reference_golden(orc, name):
    K, g = K1N_PARAMS[name]
    for key, L, rx, dec, unc in k1n_sets(name):
        got = orc.k1n_decode(K, g, rx, L)
        assert (got == dec).all(), key
        if key.endswith("p000"):
            assert (got == unc).all(), key


def test_oracle_k1n_is_the_k1_decoder_at_n2(orc):
    """n = 2: the same arithmetic as the rate-1/2 oracle, on the reference's golden frames."""
    for K in (5, 7, 9):
        for key, L, unc, rx, dec in golden_sets(K):
            assert (orc.k1n_decode(K, CODES[K], rx, L) == dec).all(), (K, key)


@pytest.mark.parametrize("name", ["k7n3", "k9n3"])
def test_n3_uint8_equals_exact_ml(orc, name):
    """For n <= 3 no uint8 sum wraps (the minimum grows by at most floor(n/2) = 1 per step,
    DESIGN.md 3), so the reference's arithmetic equals exact-metric ML (oracle_genk_decode)."""
    K, g = K1N_PARAMS[name]
    for p, seed in ((0.05, 1), (0.15, 2), (0.5, 3)):
        _, rx = k1n_frames(orc, K, g, 512, 8, p, seed, garbage=True)
        assert (orc.k1n_decode(K, g, rx, 512) == orc.genk_decode(1, K, g, rx, 512)).all(), p


def test_uint8_mode_never_wraps_differently_on_noise(orc):
    """Whether or not a code's uint8 sums can wrap (n >= 4 gives the minimum room to grow
    up to floor(n/2) per step), the drop-in decodes n != 2 with the reference's own arithmetic
    (VTB_GENK_K1_REFERENCE_U8), so parity does not depend on that bound.  On pure noise the
    K=5 rate-1/4 code stays below the wrap (no received byte is at distance 2 from every
    label), and the reference's arithmetic then equals exact ML."""
    K, g = K1N_PARAMS["k5n4"]
    _, rx = k1n_frames(orc, K, g, 1024, 32, 0.5, 9)
    assert (orc.k1n_decode(K, g, rx, 1024) == orc.genk_decode(1, K, g, rx, 1024)).all()


@pytest.mark.parametrize("L", [1, 7, 13, 100, 1001])
def test_odd_lengths_pack_like_the_reference(orc, L):
    """Any frame length (the reference pads the last byte, :226-249): error-free frames
    decode to their payload, and the n=2 case agrees with the rate-1/2 oracle."""
    K, g = K1N_PARAMS["k7n3"]
    unc, rx = k1n_frames(orc, K, g, ((L + 7) // 8) * 8, 4, 0.0, L)
    # re-encode an L-bit payload: zero the bits past L, then encode with the helper
    from helpers import encode_bits
    bits = np.unpackbits(unc, axis=1)[:, :L]
    coded = np.zeros((4, L + K - 1), np.uint8)
    for j, gj in enumerate(g):
        coded |= (encode_bits(K, (gj, gj), bits) & 1) << j
    want = np.packbits(np.concatenate([bits, np.zeros((4, (-L) % 8), np.uint8)], axis=1), axis=1)
    assert (orc.k1n_decode(K, g, coded, L) == want).all()
    assert (orc.genk_decode(1, K, g, coded, L) == want).all()
