"""K=7 and K=9 rate-1/3 hard decoding (k = 1; generators 0133 0171 0165, 0557 0663 0711) through
vtb_genk_decode_device: the K=7 pair kernel / K=9 frame kernel (k7_lds_n3, k9_n3) against the general-k kernel (VTB_KERNEL=genk), device-resident
random segments (a Viterbi decoder's work does not depend on the data), HIP events on the launch
stream.  Measurement only."""
import json
import os
import sys

import torch

sys.path.insert(0, ".")
from convolutionalencdec_amd import GenKDecoder, native  # noqa: E402

L = 1024
CODES = ((7, (0o133, 0o171, 0o165)), (9, (0o557, 0o663, 0o711)))
for K, g in CODES:
    d = GenKDecoder(1, K, g, L)
    for F in (4096, 16384, 65536):
        x = torch.randint(0, 8, (F, d.in_bytes), dtype=torch.uint8, device="cuda")
        out = torch.empty((F, d.out_bytes), dtype=torch.uint8, device="cuda")
        for arm in ("fast", "genk"):
            if arm == "genk":
                os.environ["VTB_KERNEL"] = "genk"
            else:
                os.environ.pop("VTB_KERNEL", None)
            for _ in range(3):
                d.decode_device(x, out)
            torch.cuda.synchronize()
            kern = native.last_kernel()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            steps = 20 if K == 7 or arm == "fast" else 5
            e0.record()
            for _ in range(steps):
                d.decode_device(x, out)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / steps
            print(json.dumps({"code": f"K={K} r=1/3 ({','.join(oct(v)[2:] for v in g)}) hard", "kernel": kern,
                              "frames": F, "info_bits": L, "kernel_ms": round(ms, 4),
                              "mbit_s": round(F * L / ms / 1e3, 1)}), flush=True)
        os.environ.pop("VTB_KERNEL", None)
