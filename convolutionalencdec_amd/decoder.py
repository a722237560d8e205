"""Host-side mirror of the reference decoder interface over the C ABI.

Reference (C, compile-time configured)                 here (runtime configured)
  convCodeParams.h  K, g[]                               ConvCode(K, g)
  viterbiConfigCheck()         viterbiDecoder.c:9-30     ConvCode.check()  (raises, no exit)
  viterbiInitButterflyk1()     ...Butterflyk1.c:8-44     ConvCode.edge_table()
  VITERBI_DECODER_HARD(st, coded, out, T, last=true)     ViterbiDecoder.decode(frames)
      ...Butterflyk1.c:82-263   (one frame per call)        (a batch of frames per call)
  VITERBI_DECODER_HARD(st, chunk, out, n, last=false/true) ViterbiStream.push(chunks, last)
      ...Butterflyk1.c:85-196   (state kept across calls)   (a batch of streams per call,
                                                              bits emitted once final)

`decode` takes either a torch uint8 tensor already on a ROCm device (decoded on that
device, on torch's current stream, no host round trip) or a host numpy array (copied in
and out by the C ABI).  Frames are rows: hard input [F, T] one coded segment per byte;
soft input [F, T, 2] (or [F, 2T]) 8-bit soft values.  Output: [F, ceil(L/8)] uint8,
information bits MSB-first.
"""
import ctypes
from dataclasses import dataclass

import numpy as np

from . import native

K7_CODE = (7, (0o113, 0o171))  # reference src/defaultParams/convCodeParams.c:6
K9_CODE = (9, (0o561, 0o753))  # K=9 set used by the build (SURVEY.md §8 d, config C4)


@dataclass(frozen=True)
class ConvCode:
    K: int = 7
    g: tuple = (0o113, 0o171)

    @property
    def S(self):
        return self.K - 1

    @property
    def num_states(self):
        return 1 << self.S

    def _c(self):
        return native.VtbCode.make(self.K, self.g)

    def check(self):
        c = self._c()
        native.check(native.lib().vtb_code_check(ctypes.byref(c)), f"code K={self.K} g={tuple(map(oct, self.g))}")
        return self

    def edge_table(self):
        c = self._c()
        out = np.zeros(1 << (self.K - 2), np.uint8)
        native.check(native.lib().vtb_edge_table(ctypes.byref(c), out.ctypes.data_as(ctypes.c_void_p)), "edge_table")
        return out


class ViterbiDecoder:
    """A decode plan: one code, one input format, one frame length, one device.

    The testing / measurement switches ($VTB_KERNEL, $VTB_DEBUG, $VTB_SPLIT_WARM, $VTB_SEG_*;
    csrc/vtb_internal.h Knobs) are read once, when the plan is created: setting them afterwards
    does not change an existing plan (make a new ViterbiDecoder).  GenKDecoder, which has no plan
    in the C ABI, reads them on every call."""

    def __init__(self, code=ConvCode(), frame_bits=1024, soft=False, device=0):
        self.code = code if isinstance(code, ConvCode) else ConvCode(*code)
        self.frame_bits = int(frame_bits)
        self.soft = bool(soft)
        self.device = int(device)
        self.T = self.frame_bits + self.code.S
        self.in_bytes = (2 if self.soft else 1) * self.T
        self.out_bytes = (self.frame_bits + 7) // 8
        L = native.lib()
        c = self.code._c()
        plan = ctypes.c_void_p()
        native.check(
            L.vtb_plan_create(ctypes.byref(plan), ctypes.byref(c),
                              native.VTB_INPUT_SOFT8 if self.soft else native.VTB_INPUT_HARD, self.frame_bits,
                              self.device),
            "vtb_plan_create")
        self._plan = plan

    def close(self):
        if getattr(self, "_plan", None):
            native.lib().vtb_plan_destroy(self._plan)
            self._plan = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- device-resident path ------------------------------------------------------
    def decode_device(self, frames, out=None, stream=None):
        """frames: torch uint8 tensor on this plan's device, rows of in_bytes (contiguous rows)."""
        import torch

        if frames.dtype != torch.uint8 or not frames.is_cuda:
            raise TypeError("decode_device expects a torch.uint8 tensor on a ROCm device")
        if frames.device.index != self.device:
            raise ValueError(f"frames are on {frames.device}, the plan on cuda:{self.device}")
        x = frames.reshape(frames.shape[0], -1)
        if x.shape[1] != self.in_bytes or x.stride(1) != 1:
            raise ValueError(f"expected rows of {self.in_bytes} contiguous bytes, got {tuple(x.shape)}")
        F = x.shape[0]
        if out is None:
            out = torch.empty((F, self.out_bytes), dtype=torch.uint8, device=frames.device)
        elif (out.dtype != torch.uint8 or out.device != frames.device or out.dim() != 2 or out.shape[0] < F
              or out.shape[1] < self.out_bytes or out.stride(1) != 1):
            raise ValueError(f"out must be a uint8 [>= {F}, >= {self.out_bytes}] tensor with contiguous rows on "
                             f"{frames.device}")
        if stream is None:
            stream = torch.cuda.current_stream(frames.device).cuda_stream
        native.check(
            native.lib().vtb_decode_device(self._plan, ctypes.c_void_p(x.data_ptr()), x.stride(0),
                                           ctypes.c_void_p(out.data_ptr()), out.stride(0), F, ctypes.c_void_p(stream)),
            "vtb_decode_device")
        return out

    def bind(self, frames, out, stream=None):
        """Validate (frames, out, stream) once and return a zero-argument callable that
        launches the decode of `frames` into `out` (vtb_decode_device) with no per-call
        Python checks: the repeated-batch launch of a serving loop or a bench.  `frames` must
        be contiguous (so the launcher reads the caller's own memory, never a temporary copy)
        and `out` given; the callable holds references to both, and the caller must not
        resize them while it is used."""
        import torch

        if out is None:
            raise ValueError("bind needs an output tensor")
        if not frames.is_contiguous():
            raise ValueError("bind needs contiguous frames (a reshape copy would be freed under the launcher)")
        if stream is None:
            stream = torch.cuda.current_stream(frames.device).cuda_stream
        self.decode_device(frames, out=out, stream=stream)  # validates, and warms the plan
        x = frames.reshape(frames.shape[0], -1)  # a view: frames is contiguous
        fn = native.lib().vtb_decode_device
        args = (self._plan, ctypes.c_void_p(x.data_ptr()), x.stride(0), ctypes.c_void_p(out.data_ptr()),
                out.stride(0), x.shape[0], ctypes.c_void_p(stream))
        keep = (frames, x, out)

        def launch():
            rc = fn(*args)
            if rc < 0:
                raise native.VtbError(rc, "vtb_decode_device")

        launch.tensors = keep  # the launcher owns references to the buffers it reads and writes
        return launch

    # -- host path ---------------------------------------------------------------------
    def decode_host(self, frames):
        x = np.ascontiguousarray(frames, dtype=np.uint8).reshape(-1, self.in_bytes)
        out = np.zeros((x.shape[0], self.out_bytes), np.uint8)
        native.check(
            native.lib().vtb_decode_host(self._plan, x.ctypes.data_as(ctypes.c_void_p),
                                         out.ctypes.data_as(ctypes.c_void_p), x.shape[0]),
            "vtb_decode_host")
        return out

    def decode_frame(self, frame):
        """One frame (host bytes in the plan's input layout) decoded synchronously at the lowest
        latency (vtb_decode_frame_sync); returns ceil(L/8) bytes."""
        x = np.ascontiguousarray(frame, dtype=np.uint8).reshape(-1)
        if x.size != self.in_bytes:
            raise ValueError(f"expected one frame of {self.in_bytes} bytes, got {x.size}")
        out = np.zeros(self.out_bytes, np.uint8)
        native.check(
            native.lib().vtb_decode_frame_sync(self._plan, x.ctypes.data_as(ctypes.c_void_p),
                                               out.ctypes.data_as(ctypes.c_void_p)),
            "vtb_decode_frame_sync")
        return out

    def decode(self, frames):
        try:
            import torch

            if isinstance(frames, torch.Tensor):
                return self.decode_device(frames)
        except ImportError:  # pragma: no cover
            pass
        return self.decode_host(frames)


class ViterbiStream:
    """Streaming decoder over the C ABI (vtb_stream_*; any K): `streams` independent streams
    advancing in lockstep on one device.  push(chunk, last) feeds `segments` more coded
    segments per stream (torch uint8 tensor on the device, [streams, segments] hard or
    [streams, segments, 2] / [streams, 2*segments] soft) and returns (bytes, nbits): row i of
    `bytes` holds the bits of stream i that became final in this call (MSB-first), nbits[i]
    their count (-1: window overflow, the frame is lost).  The concatenated bits of a frame
    equal ViterbiDecoder.decode of the whole frame.  last=True ends the frame."""

    def __init__(self, code=ConvCode(), streams=1, soft=False, window_steps=0, device=0):
        self.code = code if isinstance(code, ConvCode) else ConvCode(*code)
        self.streams = int(streams)
        self.soft = bool(soft)
        self.device = int(device)
        L = native.lib()
        c = self.code._c()
        h = ctypes.c_void_p()
        native.check(
            L.vtb_stream_create(ctypes.byref(h), ctypes.byref(c),
                                native.VTB_INPUT_SOFT8 if self.soft else native.VTB_INPUT_HARD, self.streams,
                                int(window_steps), self.device),
            "vtb_stream_create")
        self._h = h
        self.out_bytes = int(L.vtb_stream_out_bytes(h))

    def close(self):
        if getattr(self, "_h", None):
            native.lib().vtb_stream_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def push(self, chunk, last=False, stream=None):
        import torch

        sb = 2 if self.soft else 1
        dev = torch.device("cuda", self.device)
        if chunk is None:
            x = torch.empty((self.streams, 0), dtype=torch.uint8, device=dev)
        else:
            if chunk.dtype != torch.uint8 or not chunk.is_cuda:
                raise TypeError("push expects a torch.uint8 tensor on a ROCm device")
            if chunk.device.index != self.device:
                raise ValueError(f"chunk is on {chunk.device}, the streams on cuda:{self.device}")
            x = chunk.reshape(self.streams, -1)
            if x.stride(1) != 1:
                x = x.contiguous()
        if x.shape[1] % sb:
            raise ValueError("soft input needs two bytes per segment")
        segs = x.shape[1] // sb
        out = torch.empty((self.streams, self.out_bytes), dtype=torch.uint8, device=dev)
        nbits = torch.empty(self.streams, dtype=torch.int32, device=dev)
        if stream is None:
            stream = torch.cuda.current_stream(dev).cuda_stream
        in_ptr = ctypes.c_void_p(x.data_ptr()) if segs else None
        native.check(
            native.lib().vtb_stream_decode(self._h, in_ptr, max(x.stride(0), 1), segs, 1 if last else 0,
                                           ctypes.c_void_p(out.data_ptr()), out.stride(0),
                                           ctypes.c_void_p(nbits.data_ptr()), ctypes.c_void_p(stream)),
            "vtb_stream_decode")
        return out, nbits


def release_cached_plans():
    """Free the per-device plans decode_multi keeps between calls (vtb_release_cached_plans)."""
    native.lib().vtb_release_cached_plans()


def decode_multi(frames, code=ConvCode(), frame_bits=1024, soft=False, device_mask=0):
    """Host frames sharded across the GPUs in device_mask (vtb_decode_host_multi)."""
    code = code if isinstance(code, ConvCode) else ConvCode(*code)
    T = frame_bits + code.S
    ib = (2 if soft else 1) * T
    x = np.ascontiguousarray(frames, dtype=np.uint8).reshape(-1, ib)
    out = np.zeros((x.shape[0], (frame_bits + 7) // 8), np.uint8)
    c = code._c()
    native.check(
        native.lib().vtb_decode_host_multi(ctypes.byref(c), native.VTB_INPUT_SOFT8 if soft else native.VTB_INPUT_HARD,
                                           frame_bits, x.ctypes.data_as(ctypes.c_void_p),
                                           out.ctypes.data_as(ctypes.c_void_p), x.shape[0], device_mask),
        "vtb_decode_host_multi")
    return out


def shard_range(frames, shards, index):
    """[lo, hi) of shard `index` of `shards` over `frames` frames (vtb_shard_range)."""
    lo, hi = ctypes.c_size_t(), ctypes.c_size_t()
    native.check(native.lib().vtb_shard_range(frames, shards, index, ctypes.byref(lo), ctypes.byref(hi)),
                 "vtb_shard_range")
    return lo.value, hi.value


def decode_peer(frames, devices, code=ConvCode(), frame_bits=1024, soft=False, out=None, stage_all=False,
                stream=None):
    """Frames resident on one GPU (a torch uint8 tensor, rows of one frame) sharded across
    `devices` peer to peer over xGMI (vtb_decode_peer_multi): shards on other GPUs are copied
    there, decoded and their bytes copied back; the source GPU's own shard decodes in place.
    Asynchronous on torch's current stream of the source device."""
    import torch

    code = code if isinstance(code, ConvCode) else ConvCode(*code)
    T = frame_bits + code.S
    ib = (2 if soft else 1) * T
    x = frames.reshape(frames.shape[0], -1)
    if frames.dtype != torch.uint8 or not frames.is_cuda or x.shape[1] != ib or not x.is_contiguous():
        raise ValueError(f"frames must be a contiguous uint8 ROCm tensor of rows of {ib} bytes")
    F = x.shape[0]
    ob = (frame_bits + 7) // 8
    if out is None:
        out = torch.empty((F, ob), dtype=torch.uint8, device=frames.device)
    elif out.dtype != torch.uint8 or out.device != frames.device or tuple(out.shape) != (F, ob) or not out.is_contiguous():
        raise ValueError(f"out must be a contiguous uint8 [{F}, {ob}] tensor on {frames.device}")
    if stream is None:
        stream = torch.cuda.current_stream(frames.device).cuda_stream
    devs = (ctypes.c_int * len(devices))(*[int(d) for d in devices])
    c = code._c()
    native.check(
        native.lib().vtb_decode_peer_multi(ctypes.byref(c), native.VTB_INPUT_SOFT8 if soft else native.VTB_INPUT_HARD,
                                           frame_bits, frames.device.index, ctypes.c_void_p(x.data_ptr()),
                                           ctypes.c_void_p(out.data_ptr()), F, devs, len(devices),
                                           native.VTB_PEER_STAGE_ALL if stage_all else 0, ctypes.c_void_p(stream)),
        "vtb_decode_peer_multi")
    return out


class GenKDecoder:
    """Hard-decision decoder for a rate-k/n code (k input bits per trellis step), the
    reference's generic `viterbiDecoderHard` (src/viterbiDecoder.c:52-234) as terminated
    maximum likelihood on the GPU (vtb_genk_decode_device).  `generators` over k*K bits,
    MSB = newest input bit (src/convEncode.c conventions)."""

    def __init__(self, k, K, generators, info_bits):
        if info_bits % 8 or info_bits % k:
            raise ValueError("info_bits must be a multiple of 8 and of k (viterbiDecoder.c:222-227)")
        self.k, self.K, self.generators, self.info_bits = int(k), int(K), tuple(int(g) for g in generators), int(info_bits)
        self._code = native.VtbGenKCode.make(k, K, self.generators)
        self.in_bytes = info_bits // k + K - 1
        self.out_bytes = info_bits // 8

    def decode_device(self, frames, out=None, stream=None):
        """frames: torch uint8 tensor on a ROCm device, rows of in_bytes coded segments."""
        import torch

        if frames.dtype != torch.uint8 or not frames.is_cuda:
            raise TypeError("decode_device expects a torch.uint8 tensor on a ROCm device")
        x = frames.reshape(frames.shape[0], -1)
        if x.shape[1] != self.in_bytes or x.stride(1) != 1:
            raise ValueError(f"expected rows of {self.in_bytes} contiguous bytes, got {tuple(x.shape)}")
        F = x.shape[0]
        if out is None:
            out = torch.empty((F, self.out_bytes), dtype=torch.uint8, device=frames.device)
        elif (out.dtype != torch.uint8 or out.device != frames.device or out.dim() != 2 or out.shape[0] < F
              or out.shape[1] < self.out_bytes or out.stride(1) != 1):
            raise ValueError(f"out must be a uint8 [>= {F}, >= {self.out_bytes}] tensor with contiguous rows on "
                             f"{frames.device}")
        if stream is None:
            stream = torch.cuda.current_stream(frames.device).cuda_stream
        with torch.cuda.device(frames.device):
            native.check(
                native.lib().vtb_genk_decode_device(ctypes.byref(self._code), self.info_bits,
                                                    ctypes.c_void_p(x.data_ptr()), x.stride(0),
                                                    ctypes.c_void_p(out.data_ptr()), out.stride(0), F,
                                                    ctypes.c_void_p(stream)),
                "vtb_genk_decode_device")
        return out
