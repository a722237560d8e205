"""Synthetic frames generated on the device through the C ABI:
payload -> terminated convolutional encoding -> channel, all in HBM, so batches of any size
never cross PCIe.  The kernels live in csrc/vtb_gen.hip; their RNG stream and fixed-point
channel are specified in include/viterbi_amd.h ("Synthetic frames") and restated by the test
oracle.

Reference analogues: convEnc (src/convEncode.c:46-130) for `encode`; the harnesses' random
payloads and BSC corruption (berTestK7.c:22-43, 135-138) for `payload` / `channel`.
"""
import ctypes

from . import native


def _stream(t, stream):
    import torch

    return stream if stream is not None else torch.cuda.current_stream(t.device).cuda_stream


def _check_rows(t, min_cols, what):
    """A [rows, >= min_cols] torch.uint8 tensor on a ROCm device (the kernels read whole rows)."""
    import torch

    if not isinstance(t, torch.Tensor) or t.dtype != torch.uint8 or t.device.type != "cuda" or t.dim() != 2:
        raise TypeError(f"{what} must be a 2-D torch.uint8 tensor on a ROCm device")
    if t.shape[1] < min_cols:
        raise ValueError(f"{what} rows hold {t.shape[1]} bytes, {min_cols} needed")


def payload(frames, frame_bits, seed, device=0, stream=None):
    """[frames, ceil(L/8)] uint8 payload rows (MSB-first bits) on cuda:`device`."""
    import torch

    nb = (int(frame_bits) + 7) // 8
    out = torch.empty((int(frames), nb), dtype=torch.uint8, device=f"cuda:{device}")
    with torch.cuda.device(out.device):  # the kernels run on the current HIP device
        native.check(native.lib().vtb_payload_device(int(seed), int(frame_bits), ctypes.c_void_p(out.data_ptr()), nb,
                                                     int(frames), ctypes.c_void_p(_stream(out, stream))),
                     "vtb_payload_device")
    return out


def encode(code, frame_bits, unc, stream=None):
    """convEnc on device payload rows -> [frames, L+K-1] coded segment bytes."""
    import torch

    from .decoder import ConvCode

    code = code if isinstance(code, ConvCode) else ConvCode(*code)
    T = int(frame_bits) + code.S
    _check_rows(unc, (int(frame_bits) + 7) // 8, "encode: unc")
    out = torch.empty((unc.shape[0], T), dtype=torch.uint8, device=unc.device)
    c = code._c()
    if unc.stride(1) != 1:
        unc = unc.contiguous()
    with torch.cuda.device(unc.device):
        native.check(native.lib().vtb_encode_device(ctypes.byref(c), int(frame_bits), ctypes.c_void_p(unc.data_ptr()),
                                                    unc.stride(0), ctypes.c_void_p(out.data_ptr()), T, unc.shape[0],
                                                    ctypes.c_void_p(_stream(unc, stream))),
                     "vtb_encode_device")
    return out


def channel(coded, soft, param, seed, stream=None):
    """BSC (hard, param = p) -> [F, T] bytes, or BPSK-AWGN + 8-bit quantiser (soft, param =
    SNR dB) -> [F, T, 2] bytes."""
    import torch

    _check_rows(coded, 1, "channel: coded")
    F, T = coded.shape
    if coded.stride(1) != 1:
        coded = coded.contiguous()
    out = torch.empty((F, T, 2) if soft else (F, T), dtype=torch.uint8, device=coded.device)
    with torch.cuda.device(coded.device):
        native.check(native.lib().vtb_channel_device(native.VTB_INPUT_SOFT8 if soft else native.VTB_INPUT_HARD,
                                                     float(param), int(seed), ctypes.c_void_p(coded.data_ptr()),
                                                     coded.stride(0), T, ctypes.c_void_p(out.data_ptr()),
                                                     out.stride(0), F, ctypes.c_void_p(_stream(coded, stream))),
                     "vtb_channel_device")
    return out


def make_frames(code, frames, frame_bits, soft=True, snr_db=-5.0, p=0.0559, seed=0, device=0, stream=None):
    """(payload [F, ceil(L/8)], channel output) on the device, like synth.make_frames."""
    unc = payload(frames, frame_bits, seed, device, stream)
    coded = encode(code, frame_bits, unc, stream)
    rx = channel(coded, soft, snr_db if soft else p, seed + 1, stream)
    return unc, rx


def awgn_kq(snr_db):
    return int(native.lib().vtb_awgn_kq(float(snr_db)))


def bsc_p32(p):
    return int(native.lib().vtb_bsc_p32(float(p)))


def rand64(seed, frame, ctr):
    return int(native.lib().vtb_rand64(int(seed), int(frame), int(ctr)))
