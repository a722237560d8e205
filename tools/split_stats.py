"""Measurement only: frames per launch that the persistent split kernel could not decode split
(halves not converged within the warm-up; re-decoded by the list kernel), on device-generated
C3-shaped batches, plus the launch time.  python tools/split_stats.py [frames] [bits]"""
import ctypes
import json
import sys

import torch

sys.path.insert(0, ".")
from convolutionalencdec_amd import ConvCode, ViterbiDecoder, frames, native  # noqa: E402

F = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
L = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
lib = native.lib()
lib.vtb_debug_split_failures.restype = ctypes.c_longlong
lib.vtb_debug_split_failures.argtypes = [ctypes.c_void_p]
code = ConvCode()
for soft, param in ((True, -5.0), (True, -4.0), (True, -3.0), (False, 0.0559), (False, 0.0372), (False, 0.0226)):
    unc, rx = frames.make_frames(code, F, L, soft=soft, snr_db=param, p=param, seed=11)
    x = rx.reshape(F, -1)
    d = ViterbiDecoder(code, frame_bits=L, soft=soft)
    out = d.decode_device(x)
    torch.cuda.synchronize()
    fails = lib.vtb_debug_split_failures(d._plan)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        d.decode_device(x, out=out)
    e1.record()
    torch.cuda.synchronize()
    print(json.dumps({"soft": soft, "channel": param, "frames": F, "bits": L, "split_failures": fails,
                      "kernel_ms": round(e0.elapsed_time(e1) / 5, 4)}), flush=True)
