"""Debug helper (GPU box): decode golden sets with a forced kernel family and report the
first mismatching frames and bit positions."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
os.environ.setdefault("VTB_KERNEL", "k7")
import torch  # noqa: E402
from helpers import CODES, golden_sets  # noqa: E402

from convolutionalencdec_amd import ConvCode, ViterbiDecoder  # noqa: E402

K = 7
for key, L, unc, rx, dec in golden_sets(K):
    d = ViterbiDecoder(ConvCode(K, CODES[K]), frame_bits=L)
    x = torch.from_numpy(np.ascontiguousarray(rx).reshape(rx.shape[0], -1)).cuda()
    out = d.decode_device(x).cpu().numpy()
    bad = np.nonzero((out != dec).any(axis=1))[0]
    print(key, rx.shape, "bad frames", len(bad), bad[:10])
    for f in bad[:3]:
        idx = np.nonzero(np.unpackbits(out[f] ^ dec[f]))[0]
        print("   frame", f, "bad bits", len(idx), idx[:30], "rx high bits", int((rx[f] >> 2).any()))

if len(sys.argv) > 1:
    from helpers import Oracle, random_frames

    orc = Oracle()
    for F in (4, 32, 33):
        unc, rx = random_frames(orc, K, 1024, F, 0.0, 5)
        d = ViterbiDecoder(ConvCode(K, CODES[K]), frame_bits=1024)
        x = torch.from_numpy(np.ascontiguousarray(rx).reshape(rx.shape[0], -1)).cuda()
        out = d.decode_device(x).cpu().numpy()
        bad = np.nonzero((out != unc).any(axis=1))[0]
        print("random F", F, "bad frames", len(bad), bad[:10])
    key, L, unc, rx, dec = next(iter(golden_sets(K)))
    print("golden first set", key, "unc==dec", bool((unc == dec).all()), "uncoded last bytes", unc[0, -2:], dec[0, -2:])
