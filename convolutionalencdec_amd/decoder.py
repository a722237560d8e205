"""Host-side mirror of the reference decoder interface over the C ABI.

Reference (C, compile-time configured)                 here (runtime configured)
  convCodeParams.h  K, g[]                               ConvCode(K, g)
  viterbiConfigCheck()         viterbiDecoder.c:9-30     ConvCode.check()  (raises, no exit)
  viterbiInitButterflyk1()     ...Butterflyk1.c:8-44     ConvCode.edge_table()
  VITERBI_DECODER_HARD(st, coded, out, T, last=true)     ViterbiDecoder.decode(frames)
      ...Butterflyk1.c:82-263   (one frame per call)        (a batch of frames per call)

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
    """A decode plan: one code, one input format, one frame length, one device."""

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
        x = frames.reshape(frames.shape[0], -1)
        if x.shape[1] != self.in_bytes or x.stride(1) != 1:
            raise ValueError(f"expected rows of {self.in_bytes} contiguous bytes, got {tuple(x.shape)}")
        F = x.shape[0]
        if out is None:
            out = torch.empty((F, self.out_bytes), dtype=torch.uint8, device=frames.device)
        if stream is None:
            stream = torch.cuda.current_stream(frames.device).cuda_stream
        native.check(
            native.lib().vtb_decode_device(self._plan, ctypes.c_void_p(x.data_ptr()), x.stride(0),
                                           ctypes.c_void_p(out.data_ptr()), out.stride(0), F, ctypes.c_void_p(stream)),
            "vtb_decode_device")
        return out

    # -- host path ---------------------------------------------------------------------
    def decode_host(self, frames):
        x = np.ascontiguousarray(frames, dtype=np.uint8).reshape(-1, self.in_bytes)
        out = np.zeros((x.shape[0], self.out_bytes), np.uint8)
        native.check(
            native.lib().vtb_decode_host(self._plan, x.ctypes.data_as(ctypes.c_void_p),
                                         out.ctypes.data_as(ctypes.c_void_p), x.shape[0]),
            "vtb_decode_host")
        return out

    def decode(self, frames):
        try:
            import torch

            if isinstance(frames, torch.Tensor):
                return self.decode_device(frames)
        except ImportError:  # pragma: no cover
            pass
        return self.decode_host(frames)


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
