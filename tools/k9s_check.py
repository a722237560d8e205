"""K=9 one-frame-per-wave kernel (k9s): bit-exactness against the oracle on a
spread of shapes (odd / even T, short / long frames, 1 to 24,576 frames, clean to pure noise,
soft and hard), with the completeness guards shipped and forced, the pair kernel (VTB_DEBUG bit
18) beside it.  Measurement / bring-up script; the suite's own cases are in tests/.

    python tools/k9s_check.py            # prints one line per case, exits 1 on any mismatch
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402
from helpers import CODES, Oracle, random_frames  # noqa: E402

from convolutionalencdec_amd import ConvCode, ViterbiDecoder, native  # noqa: E402

PAIR = 1 << 18
CAP = 1 << 17


def frames(orc, L, F, soft, noise, seed):
    if soft:
        sigma = {0.0: 0.3, 0.03: 0.56, 0.07: 0.7, 0.5: 4.0}[noise]
        _, x = random_frames(orc, 9, L, F, 0.0, seed, soft=True, sigma=sigma)
    else:
        _, x = random_frames(orc, 9, L, F, noise, seed)
    return np.ascontiguousarray(x).reshape(F, -1)


def main():
    orc = Oracle()
    cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
    native.set_guard_counter(cnt.data_ptr())
    cases = [(1024, 64, True, 0.07), (1024, 64, False, 0.07), (1001, 33, False, 0.5), (1001, 33, True, 0.5),
             (1, 3, False, 0.0), (8, 5, True, 0.0), (57, 7, True, 0.03), (200, 65, False, 0.03),
             (1024, 4096, False, 0.03), (1024, 4096, True, 0.07), (4095, 40, True, 0.07), (16384, 6, False, 0.07),
             (16383, 5, True, 0.5), (512, 24576, False, 0.07), (2048, 9001, True, 0.5), (3, 2, True, 0.5)]
    fails = 0
    for i, (L, F, soft, noise) in enumerate(cases):
        x = frames(orc, L, F, soft, noise, 3000 + i)
        want = orc.decode(9, CODES[9], x, L, soft=soft, threads=16)
        xd = torch.from_numpy(x).cuda()
        for dbg in (0, CAP, PAIR):
            os.environ["VTB_DEBUG"] = str(dbg)
            cnt.zero_()
            d = ViterbiDecoder(ConvCode(9, CODES[9]), frame_bits=L, soft=soft)
            got = d.decode_device(xd).cpu().numpy()
            torch.cuda.synchronize()
            bad = np.flatnonzero((got != want).any(axis=1))
            fails += bad.size > 0
            print(f"L={L} F={F} soft={soft} noise={noise} dbg={dbg}: kernel {native.last_kernel()} "
                  f"bad {bad.size} first {bad[:4].tolist()} guard {int(cnt.item())}", flush=True)
    native.set_guard_counter(0)
    print("FAILS", fails)
    sys.exit(1 if fails else 0)


if __name__ == "__main__":
    main()
