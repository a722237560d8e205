"""Device frame generator (csrc/vtb_gen.hip) -- CPU side: the oracle's
restatement is pinned (encoder against the reference's golden frames, RNG and fixed-point
constants against the library's host exports, channel statistics), so the GPU tests in
test_gpu_frames.py can compare the kernels with it byte for byte."""
import math

import numpy as np
import pytest

from helpers import CODES, Oracle, encode_bits, golden_sets

from convolutionalencdec_amd import frames, synth


@pytest.fixture(scope="module")
def orc():
    return Oracle()


def test_rand64_matches_library(orc):
    for seed, f, c in [(0, 0, 0), (1, 2, 3), (314, 4095, 8 * 1029 + 7), (2**63 + 5, 2**40, 2**33)]:
        assert orc.rand64(seed, f, c) == frames.rand64(seed, f, c)
    # pinned value of the specified stream (include/viterbi_amd.h)
    assert frames.rand64(1, 2, 3) == 0xB28AD7CBCB6754BF


def test_fixed_point_constants(orc):
    for snr in (-5.0, -4.0, -3.0, 0.0, 6.5):
        assert orc.L.oracle_awgn_kq(snr) == frames.awgn_kq(snr)
        assert frames.awgn_kq(snr) == round(synth.sigma_for_snr(snr) * 127.5 * 65536)
    for p in (0.0, 1e-6, 0.0559, 0.5, 1.0):
        assert orc.L.oracle_bsc_p32(p) == frames.bsc_p32(p)
    assert frames.bsc_p32(0.5) == 2**31


@pytest.mark.parametrize("K", [5, 7, 9])
def test_encoder_matches_reference_golden(orc, K):
    """Error-free golden sets (p = 0) were produced by the reference encoder itself."""
    for key, L, unc, rx, _ in golden_sets(K):
        if not key.endswith("p000"):
            continue
        assert (orc.gen_encode(K, CODES[K], L, unc) == rx).all(), key


@pytest.mark.parametrize("L", [1, 7, 8, 13, 100, 1024])
def test_encoder_arbitrary_length(orc, L):
    rng = np.random.default_rng(L)
    unc = rng.integers(0, 256, (5, (L + 7) // 8), dtype=np.uint8)
    bits = np.unpackbits(unc, axis=1)[:, :L]
    for K in (3, 7, 9):
        g = CODES.get(K, (0o7, 0o5))
        assert (orc.gen_encode(K, g, L, unc) == encode_bits(K, g, bits)).all()


def test_payload_spec(orc):
    out = orc.gen_payload(9865, 1021, 3)
    assert out.shape == (3, 128)
    assert out[2, 9] == (orc.rand64(9865, 2, 1) >> 8) & 0xFF
    assert out[0, 127] & 0x07 == 0  # 1021 bits: three pad bits cleared
    assert out[0, 127] == (orc.rand64(9865, 0, 15) >> 56) & 0xF8


def test_bsc_statistics(orc):
    coded = np.zeros((64, 1030), np.uint8)
    for p in (0.0, 0.0559, 0.5):
        rx = orc.gen_bsc(7, frames.bsc_p32(p), coded)
        rate = np.unpackbits(rx[..., None], axis=-1)[..., -2:].mean()
        assert abs(rate - p) < 4 * math.sqrt(max(p * (1 - p), 1e-9) / rx.size / 2) + 1e-12


def test_awgn_statistics(orc):
    """Quantised channel statistics match the float model q = clamp(round((1 - y) * 127.5))
    with y ~ N(1 - 2b, sigma) (synth.soft_awgn): mean and spread of q and the hard-slice
    BER, for both transmitted bits."""
    snr = -3.0
    sigma = synth.sigma_for_snr(snr)
    coded = np.tile(np.array([0, 3], np.uint8), (128, 515))
    q = orc.gen_awgn8(11, frames.awgn_kq(snr), coded).astype(np.float64)
    ref = synth.soft_awgn(coded, snr, 5).astype(np.float64)
    for b in (0, 1):
        qb, rb = q[:, b::2].reshape(-1), ref[:, b::2].reshape(-1)
        assert abs(qb.mean() - rb.mean()) < 1.0
        assert abs(qb.std() - rb.std()) / rb.std() < 0.03
        ber = ((qb >= 128) != b).mean()
        assert abs(ber - 0.5 * math.erfc(1 / sigma / math.sqrt(2))) < 0.004


def test_device_generators_reject_bad_rows():
    """encode / channel validate their inputs on the host before any launch (a short row
    would make the kernel read past it)."""
    import torch

    from convolutionalencdec_amd.decoder import ConvCode

    with pytest.raises(TypeError):
        frames.encode(ConvCode(), 1024, torch.zeros((2, 128), dtype=torch.uint8))  # host tensor
    with pytest.raises(TypeError):
        frames.encode(ConvCode(), 1024, np.zeros((2, 128), dtype=np.uint8))
    with pytest.raises(TypeError):
        frames.channel(torch.zeros((2, 1030), dtype=torch.int32), True, -5.0, 1)
