import json, os, sys
import torch
sys.path.insert(0, ".")
from convolutionalencdec_amd import GenKDecoder, native
L = 1024
d = GenKDecoder(1, 7, (0o133, 0o171, 0o165), L)
for F in (1000, 2048, 3072, 3584, 4096, 6144, 7168, 14336, 28672):
    x = torch.randint(0, 8, (F, d.in_bytes), dtype=torch.uint8, device="cuda")
    out = torch.empty((F, d.out_bytes), dtype=torch.uint8, device="cuda")
    for _ in range(3):
        d.decode_device(x, out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        d.decode_device(x, out)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    print(json.dumps({"F": F, "kernel": native.last_kernel(), "us": round(ms * 1e3, 1), "gbit_s": round(F * L / ms / 1e6, 1)}), flush=True)
