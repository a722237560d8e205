"""Measurement/debug only: replay one streaming fuzz case (tests/test_gpu_fuzz.py
test_stream_random_chunking_vs_oracle) and report, per stream, the first bit that differs from
the oracle's whole-frame decode and the call that emitted it; then the same frame pushed whole.

    python tools/dbg_stream_case.py 20
"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    import torch

    import test_gpu_fuzz as tf
    from helpers import CODES, Oracle, random_frames

    from convolutionalencdec_amd import ConvCode, ViterbiStream

    orc = Oracle()
    cases = {c[0]: c for c in tf._stream_cases()}
    i, K, L, F, soft, noise = cases[int(sys.argv[1])]
    g = CODES[K]
    sb = 2 if soft else 1
    T = L + K - 1
    for mode in ("fuzz chunking", "whole frame", "fuzz chunking again"):
        rng = np.random.default_rng(4000 + i)
        vs = ViterbiStream(ConvCode(K, g), streams=F, soft=soft)
        for frame in range(1):
            if soft:
                sigma = {0.0: 0.3, 0.03: 0.56, 0.07: 0.7, 0.5: 4.0}[noise]
                unc, x = random_frames(orc, K, L, F, 0.0, 3000 + 2 * i + frame, soft=True, sigma=sigma)
            else:
                unc, x = random_frames(orc, K, L, F, noise, 3000 + 2 * i + frame)
            x = np.ascontiguousarray(x).reshape(F, -1)
            want = np.unpackbits(orc.decode(K, g, x, L, soft=soft, threads=16), axis=1)[:, :L]
            xd = torch.from_numpy(x).cuda()
            got = [[] for _ in range(F)]
            calls = []
            pos = 0
            while True:
                c = int(min(T - pos, rng.integers(0, 1201))) if mode != "whole frame" else T
                last = pos + c == T
                out, nb = vs.push(xd[:, pos * sb:(pos + c) * sb] if c else None, last=last)
                pos += c
                out, nb = out.cpu().numpy(), nb.cpu().numpy()
                calls.append((pos, c, nb.tolist()))
                for f in range(F):
                    if nb[f] > 0:
                        got[f].append(np.unpackbits(out[f])[:nb[f]])
                if last:
                    break
            res = []
            for f in range(F):
                bits = np.concatenate(got[f]) if got[f] else np.zeros(0, np.uint8)
                bad = np.flatnonzero(bits[:L] != want[f][:bits.size]) if bits.size else np.zeros(0, int)
                first = int(bad[0]) if bad.size else None
                # which call emitted the first bad bit
                who = None
                if first is not None:
                    acc = 0
                    for k, (p, c, nb) in enumerate(calls):
                        acc += max(nb[f], 0)
                        if acc > first:
                            who = k
                            break
                res.append({"stream": f, "bits": int(bits.size), "n_bad": int(bad.size), "first_bad": first,
                            "last_bad": int(bad[-1]) if bad.size else None, "call": who})
            print(json.dumps({"mode": mode, "case": [i, K, L, F, soft, noise], "calls": calls if mode != "whole frame" else len(calls),
                              "streams": res}), flush=True)


if __name__ == "__main__":
    main()
