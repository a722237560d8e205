"""GPU: BASELINE config C3 at full size -- 65536 x 2048-bit K=7 frames per SNR point, made
on the device (payload, encoder, channel: csrc/vtb_gen.hip), decoded on the GPU and checked
against the oracle on the WHOLE batch, bit for bit; then the decoded bit-error rates against
the reference's own berTestK7 known answer at the same channel points.

berTestK7 (berTestK7.c:95-100) decodes 10000 x 2048-bit hard frames per point
through a BSC with p = 5.5856e-2 / 3.7162e-2 / 2.2622e-2, the hard slices of BPSK-AWGN at
SNR -5 / -4 / -3 dB (SURVEY.md §8 d), and counts 92418 / 9655 / 655 decoded bit errors.
The device BSC draws its flips from a counter-based RNG, not glibc rand(), so the hard
counts here are a different sample of the same channel.  They come out 5.0 / 7.0 / 0.1 %
below the reference's: its glibc TYPE_3 generator (r[i] = r[i-3] + r[i-31]) gives slightly
heavier tails of clustered flips (P(>= 6 flips in a 35-bit window) 2.5-3 % above the
binomial's at the first two points, measured on the reference's stream with the oracle's
restatement of it), and clusters are what the decoder fails on; ten-thousand-frame
sub-batches of this run spread by only 0.6 / 2.3 / 6.9 %.  So the band is +-12 %, and the
exact pin of the reference's counts is the replay of its own stream
(test_gpu_parity.py::test_bertest_k7_kat_on_gpu).  Soft decoding of the
AWGN channel at the same SNR must beat hard decoding (parity for soft is pinned by the
oracle, since the reference has no soft decoder)."""
import os

import numpy as np
import pytest

from helpers import BERTEST_ERRORS, BERTEST_P, CODES, Oracle

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from convolutionalencdec_amd import ConvCode, ViterbiDecoder, frames, native  # noqa: E402

K, L, F = 7, 2048, 65536
SNRS = (-5.0, -4.0, -3.0)
REF_BITS = 10000 * 2048  # berTestK7: 10000 packets of 256 bytes per point
BAND = 0.12  # relative, see the module docstring
THREADS = min(16, os.cpu_count() or 1)


@pytest.fixture(scope="module")
def orc():
    return Oracle()


@pytest.fixture(scope="module", autouse=True)
def gpu_present():
    if not torch.cuda.is_available() or native.lib().vtb_device_count() < 1:
        pytest.fail("no gfx950 GPU visible to the C ABI (GPU tests must not silently pass)")


def _run(orc, soft, c):
    code = ConvCode(K, CODES[K])
    unc, rx = frames.make_frames(code, F, L, soft=soft, snr_db=SNRS[c], p=BERTEST_P[c], seed=9865 + 17 * c)
    dec = ViterbiDecoder(code, frame_bits=L, soft=soft)
    out = dec.decode_device(rx.reshape(F, -1)).cpu().numpy()
    rx_h = rx.reshape(F, -1).cpu().numpy()
    ref = orc.decode(K, CODES[K], rx_h, L, soft=soft, threads=THREADS)
    mism = np.flatnonzero((out != ref).any(axis=1))
    assert mism.size == 0, f"{mism.size} of {F} frames differ from the oracle (first {mism[:8]})"
    return int(np.unpackbits(out ^ unc.cpu().numpy()).sum())


@pytest.mark.parametrize("c", [0, 1, 2])
def test_c3_full_batch_bit_exact_and_ber(orc, c):
    hard_err = _run(orc, False, c)
    soft_err = _run(orc, True, c)
    ref_rate = BERTEST_ERRORS[c] / REF_BITS
    rate = hard_err / (F * L)
    assert abs(rate / ref_rate - 1.0) < BAND, (c, rate, ref_rate)
    # 8-bit soft decoding of the unsliced channel gains ~2 dB: far fewer errors
    assert soft_err < 0.25 * hard_err, (c, soft_err, hard_err)
    print(f"SNR {SNRS[c]:+.0f} dB: hard BER {rate:.3e} (reference berTestK7 {ref_rate:.3e}), "
          f"soft BER {soft_err / (F * L):.3e}")
