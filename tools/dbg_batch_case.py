"""Measurement/debug only: replay batch fuzz cases (tests/test_gpu_fuzz.py
test_random_case_vs_oracle, VTB_FUZZ_N / VTB_FUZZ_SEED as in the sweep) through several kernel
choices and report the frames that differ from the oracle.

    VTB_FUZZ_N=2000 VTB_FUZZ_SEED=31337 python tools/dbg_batch_case.py 1173 1833
"""
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    import torch

    import test_gpu_fuzz as tf  # the sweep's case generator (test infrastructure)
    from helpers import CODES, Oracle, random_frames

    from convolutionalencdec_amd import ConvCode, ViterbiDecoder, native

    orc = Oracle()
    cases = {c[0]: c for c in tf._cases()}
    lib = native.lib()
    lib.vtb_debug_split_failures.restype = ctypes.c_longlong
    lib.vtb_debug_split_failures.argtypes = [ctypes.c_void_p]
    for idx in [int(v) for v in sys.argv[1:]]:
        i, K, L, F, soft, noise, strided = cases[idx]
        g = tf.K3 if K == 3 else CODES[K]
        if soft:
            sigma = {0.0: 0.3, 0.03: 0.56, 0.07: 0.7, 0.5: 4.0}[noise]
            unc, x = random_frames(orc, K, L, F, 0.0, 1000 + i, soft=True, sigma=sigma, g=g)
        else:
            unc, x = random_frames(orc, K, L, F, noise, 1000 + i, g=g)
        x = np.ascontiguousarray(x).reshape(F, -1)
        want = orc.decode(K, g, x, L, soft=soft, threads=16)
        xd = torch.from_numpy(x).cuda()
        for label, env in (("default", {}), ("default again", {}), ("no split loop", {"VTB_DEBUG": "4096"}),
                           ("split loop, warm-up 48", {"VTB_SPLIT_WARM": "48"}),
                           ("split loop, warm-up 144", {"VTB_SPLIT_WARM": "144"}),
                           ("first 4096 frames", {}), ("the bad frames alone", {})):
            saved = {k: os.environ.get(k) for k in env}
            os.environ.update(env)
            try:
                d = ViterbiDecoder(ConvCode(K, g), frame_bits=L, soft=soft)
                if label == "first 4096 frames":
                    sel = np.arange(min(F, 4096))
                elif label == "the bad frames alone":
                    sel = bad0 if bad0.size else np.arange(1)
                else:
                    sel = np.arange(F)
                got = d.decode_device(xd[torch.from_numpy(sel).cuda()].contiguous()).cpu().numpy()
                fails = lib.vtb_debug_split_failures(d._plan)
                d.close()
            finally:
                for k, v in saved.items():
                    if v is None:
                        os.environ.pop(k, None)
                    else:
                        os.environ[k] = v
            bad = sel[np.flatnonzero((got != want[sel]).any(axis=1))]
            if label == "default":
                bad0 = bad
            nbits = [int((np.unpackbits(got[list(sel).index(b)]) != np.unpackbits(want[b])).sum()) for b in bad[:4]]
            print(json.dumps({"case": idx, "K": K, "L": L, "F": F, "soft": soft, "noise": noise, "strided": strided,
                              "path": label, "split_list_frames": fails, "bad_frames": bad[:8].tolist(),
                              "n_bad": int(bad.size), "bad_bits": nbits}), flush=True)


if __name__ == "__main__":
    main()
