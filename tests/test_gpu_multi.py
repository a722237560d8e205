"""GPU: the multi-GPU paths on one MI355X, and BASELINE config C5's per-GPU shard.

* vtb_decode_peer_multi (device-sourced sharding over xGMI, SURVEY.md §8 e): on one GPU the
  shards of a listed source device decode in place, and with VTB_PEER_STAGE_ALL every shard
  goes through its own buffers with peer-copy calls (device to itself here), exercising the
  scatter, the per-shard plans and streams and the gather.  Every result must equal the
  single-plan decode bit for bit.  With two or more GPUs the real peer test runs too.
* vtb_decode_host_multi on uneven shard counts.
* C5: 2^20 frames over 8 GPUs is 131,072 x 1,024-bit soft frames per GPU; one GPU's shard is
  generated on the device, decoded, and compared with the oracle on the WHOLE shard."""
import os

import numpy as np
import pytest

from helpers import CODES, Oracle

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from convolutionalencdec_amd import (ConvCode, ViterbiDecoder, decode_multi, decode_peer, frames,  # noqa: E402
                                     native, release_cached_plans)

THREADS = min(16, os.cpu_count() or 1)


@pytest.fixture(scope="module")
def orc():
    return Oracle()


@pytest.fixture(scope="module", autouse=True)
def gpu_present():
    if not torch.cuda.is_available() or native.lib().vtb_device_count() < 1:
        pytest.fail("no gfx950 GPU visible to the C ABI (GPU tests must not silently pass)")
    yield
    release_cached_plans()


def _frames(K, F, L, soft, seed):
    code = ConvCode(K, CODES[K])
    unc, rx = frames.make_frames(code, F, L, soft=soft, snr_db=-4.0, p=0.04, seed=seed)
    return code, unc, rx.reshape(F, -1).contiguous()


def _direct(code, rx, L, soft):
    out = ViterbiDecoder(code, frame_bits=L, soft=soft).decode_device(rx)
    torch.cuda.synchronize()
    return out.cpu()


@pytest.mark.parametrize("soft", [False, True])
@pytest.mark.parametrize("K,L,F", [(7, 1024, 1001), (7, 4000, 333), (9, 1024, 257), (5, 100, 64)])
def test_peer_in_place_single_device(K, L, F, soft):
    code, unc, rx = _frames(K, F, L, soft, seed=F + L)
    want = _direct(code, rx, L, soft)
    got = decode_peer(rx, [0], code, L, soft)
    torch.cuda.synchronize()
    assert torch.equal(got.cpu(), want)


@pytest.mark.parametrize("soft", [False, True])
@pytest.mark.parametrize("K,L,F,devs", [(7, 1024, 1001, [0, 0, 0]), (7, 2048, 4099, [0, 0]), (9, 512, 77, [0, 0, 0, 0]),
                                        (7, 1024, 2, [0, 0, 0])])
def test_peer_staged_shards(K, L, F, devs, soft):
    """Every shard through its own buffers: scatter copy, decode on the shard's stream and plan,
    gather copy; uneven F / G and more shards than frames."""
    code, unc, rx = _frames(K, F, L, soft, seed=3 * F + K)
    want = _direct(code, rx, L, soft)
    got = decode_peer(rx, devs, code, L, soft, stage_all=True)
    torch.cuda.synchronize()
    assert torch.equal(got.cpu(), want)
    # repeated call on the kept contexts, with a different batch
    code, unc, rx2 = _frames(K, F, L, soft, seed=3 * F + K + 1)
    got2 = decode_peer(rx2, devs, code, L, soft, stage_all=True)
    torch.cuda.synchronize()
    assert torch.equal(got2.cpu(), _direct(code, rx2, L, soft))


def test_peer_orders_after_the_callers_stream():
    """The shards start after the caller's queued work: frames written on the caller's stream
    right before the call are the ones decoded."""
    code, unc, rx = _frames(7, 2048, 1024, True, seed=11)
    want = _direct(code, rx, 1024, True)
    s = torch.cuda.Stream()
    dst = torch.zeros_like(rx)
    with torch.cuda.stream(s):
        torch.cuda._sleep(2_000_000)  # keep the stream busy, then write the frames
        dst.copy_(rx)
        out = decode_peer(dst, [0, 0], code, 1024, True, stage_all=True)
    s.synchronize()
    assert torch.equal(out.cpu(), want)


def test_peer_bad_device():
    code, unc, rx = _frames(7, 16, 1024, False, seed=1)
    n = torch.cuda.device_count()
    with pytest.raises(native.VtbError) as e:
        decode_peer(rx, [0, n], code, 1024, False)
    assert e.value.code == native.VTB_ERR_DEVICE


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs two GPUs (real xGMI peers)")
def test_peer_two_gpus():
    code, unc, rx = _frames(7, 8192, 1024, True, seed=21)
    want = _direct(code, rx, 1024, True)
    for devs in ([0, 1], [1, 0], [0, 1, 1, 0]):
        got = decode_peer(rx, devs, code, 1024, True)
        torch.cuda.synchronize()
        assert torch.equal(got.cpu(), want), devs


def test_host_multi_uneven():
    code, unc, rx = _frames(7, 1001, 1024, True, seed=5)
    want = _direct(code, rx, 1024, True).numpy()
    got = decode_multi(rx.cpu().numpy(), code, 1024, True, device_mask=0)
    assert (got == want).all()


def test_c5_per_gpu_shard_whole_batch(orc):
    """BASELINE C5 per GPU: 131,072 x 1,024-bit K=7 soft frames (2^20 over 8 GPUs) from the
    device generator, decoded on the GPU and compared with the oracle on every frame; and the
    same shard through the peer path as two staged shards."""
    F, L = 131072, 1024
    code = ConvCode(7, CODES[7])
    unc, rx = frames.make_frames(code, F, L, soft=True, snr_db=-5.0, seed=2 ** 20)
    rx = rx.reshape(F, -1).contiguous()
    out = ViterbiDecoder(code, frame_bits=L, soft=True).decode_device(rx)
    peer = decode_peer(rx, [0, 0], code, L, True, stage_all=True)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    ref = orc.decode(7, CODES[7], rx.cpu().numpy(), L, soft=True, threads=THREADS)
    mism = np.flatnonzero((got != ref).any(axis=1))
    assert mism.size == 0, f"{mism.size} of {F} frames differ from the oracle (first {mism[:8]})"
    assert (peer.cpu().numpy() == got).all()
    ber = float(np.unpackbits(got ^ unc.cpu().numpy()).mean())
    assert ber < 1e-3, ber
