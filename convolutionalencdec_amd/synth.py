"""Seeded synthetic frames for bench.py and smoke(): payload -> terminated convolutional
encoding -> channel.  Host-side data generation (plumbing, not the measured path).

Encoding follows the reference encoder semantics (src/convEncode.c:46-130: MSB-first
payload, newest bit in the shift-register LSB, generator i -> bit i of each segment byte,
K-1 zero tail segments).  Channels (SURVEY.md §8 d):
  BSC       each coded bit flipped with probability p (berTestK7.c:29-43)
  AWGN      BPSK 0 -> +1, 1 -> -1, sigma = sqrt(1 / (2 Es/N0)), Es/N0 = SNR + 10 log10(4)
            (4 samples per symbol as berTestK7's SNR column), then the 8-bit soft quantiser
            q = clamp(round((1 - y) / 2 * 255), 0, 255)  (0 = confident 0, 255 = confident 1)
"""
import math

import numpy as np


def sigma_for_snr(snr_db, samples_per_symbol=4):
    esn0 = 10.0 ** ((snr_db + 10.0 * math.log10(samples_per_symbol)) / 10.0)
    return math.sqrt(1.0 / (2.0 * esn0))


def encode_bits(K, g, bits):
    """Terminated rate-1/2 encoding of bit rows [F, L] -> coded segments [F, L+K-1] uint8."""
    bits = np.asarray(bits, np.uint8)
    F, L = bits.shape
    S = K - 1
    padded = np.concatenate([np.zeros((F, S), np.uint8), bits, np.zeros((F, S), np.uint8)], axis=1)
    T = L + S
    out = np.zeros((F, T), np.uint8)
    for j, gj in enumerate(g):
        acc = np.zeros((F, T), np.uint8)
        for i in range(K):  # tap i = input i steps ago = bit K-1-i of the Proakis generator
            if (gj >> (K - 1 - i)) & 1:
                acc ^= padded[:, S - i:S - i + T]
        out |= (acc << j).astype(np.uint8)
    return out


def payload(frames, frame_bits, seed):
    rng = np.random.default_rng(seed)
    nb = (frame_bits + 7) // 8
    unc = rng.integers(0, 256, (frames, nb), dtype=np.uint8)
    if frame_bits % 8:
        unc[:, -1] &= np.uint8((0xFF << (8 - frame_bits % 8)) & 0xFF)
    return unc


def soft_awgn(coded, snr_db, seed):
    rng = np.random.default_rng(seed)
    b = np.stack([coded & 1, (coded >> 1) & 1], axis=-1).astype(np.float32)
    y = (1.0 - 2.0 * b) + np.float32(sigma_for_snr(snr_db)) * rng.standard_normal(b.shape, dtype=np.float32)
    return np.clip(np.rint((1.0 - y) * 127.5), 0, 255).astype(np.uint8)


def hard_bsc(coded, p, seed):
    rng = np.random.default_rng(seed)
    flips = (rng.random(coded.shape + (2,)) < p).astype(np.uint8)
    return (coded ^ (flips[..., 0] | (flips[..., 1] << 1))).astype(np.uint8)


def make_frames(K, g, frames, frame_bits, soft=True, snr_db=-5.0, p=0.0559, seed=0):
    """Returns (payload bytes [F, ceil(L/8)], channel output: soft [F, T, 2] or hard [F, T])."""
    unc = payload(frames, frame_bits, seed)
    coded = encode_bits(K, g, np.unpackbits(unc, axis=1)[:, :frame_bits])
    rx = soft_awgn(coded, snr_db, seed + 1) if soft else hard_bsc(coded, p, seed + 1)
    return unc, rx
