"""Generic-kernel timing sweep (vtb_lds_path.hip): LDS variant against the global-survivor (GS)
variant, by K, frame length and input kind, in one process.  Measurement only.

Frames come from the device generator (vtb_payload / encode / channel kernels); every plan is
created with the VTB_DEBUG value of its row (knobs are read at plan creation), timed over
`--reps` back-to-back launches with HIP events on the launch stream, the GS and LDS rows
interleaved.  Prints one JSON line per (K, L, soft, variant): microseconds per launch, decoded
Gbit/s and the kernel instance that ran.  Rows whose LDS variant does not fit one CU are GS only.

usage: python tools/generic_sweep.py [--frames F] [--reps R] [--K 3,5,6,8] [--L 1024,4096,9000,16384]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

GS_BIT = 1 << 19


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--K", default="3,4,5,6,8")
    ap.add_argument("--L", default="1024,4096,9000,16384")
    ap.add_argument("--rounds", type=int, default=2)
    args = ap.parse_args()
    import torch

    from bench import CODES
    from convolutionalencdec_amd import ConvCode, ViterbiDecoder, native
    from convolutionalencdec_amd import frames as devframes

    dev = torch.device("cuda", 0)
    for K in map(int, args.K.split(",")):
        code = ConvCode(*CODES[K])
        for L in map(int, args.L.split(",")):
            for soft in (False, True):
                _, rx = devframes.make_frames(code, args.frames, L, soft=soft, snr_db=-4.0, p=0.04, seed=K + L,
                                              device=0)
                x = rx.reshape(args.frames, -1)
                res = {}
                for rnd in range(args.rounds):
                    for dbg in (0, GS_BIT):
                        os.environ["VTB_DEBUG"] = str(dbg)
                        d = ViterbiDecoder(code, frame_bits=L, soft=soft)
                        out = d.decode_device(x)
                        kern = native.last_kernel()
                        if dbg == 0 and kern == "lds_path_gs":
                            d.close()
                            continue  # the LDS variant does not fit: the GS row is the default
                        s = torch.cuda.current_stream(dev)
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        torch.cuda.synchronize()
                        e0.record(s)
                        for _ in range(args.reps):
                            d.decode_device(x, out=out)
                        e1.record(s)
                        e1.synchronize()
                        us = e0.elapsed_time(e1) * 1000.0 / args.reps
                        res.setdefault(kern, []).append(us)
                        d.close()
                for kern, v in res.items():
                    best = min(v)
                    print(json.dumps({"K": K, "L": L, "soft": soft, "kernel": kern, "frames": args.frames,
                                      "us": [round(u, 1) for u in v],
                                      "gbps": round(args.frames * L / best / 1e3, 2)}), flush=True)
    os.environ.pop("VTB_DEBUG", None)


if __name__ == "__main__":
    main()
