"""Measurement only: per-wave phase timestamps of the K=7 frame kernel (Launch::tstamp).

    python tools/tstamp.py [--frames F] [--frame-bits L] [--hard] [--reps N]

Runs N back-to-back launches of the bench workload and stamps the middle one (realtime
100 MHz counter at entry / after the ACS / after the traceback / at exit, shader clock at
entry and exit, HW_ID, XCC_ID per wave).  Prints the launch's wave start ramp, phase
durations and effective clock.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=4096)
    ap.add_argument("--frame-bits", type=int, default=1024)
    ap.add_argument("--hard", action="store_true")
    ap.add_argument("--reps", type=int, default=21)
    ap.add_argument("--json", default="")
    ap.add_argument("--raw", default="", help="save the raw per-wave stamps (.npy)")
    a = ap.parse_args()
    import torch

    from convolutionalencdec_amd import ConvCode, ViterbiDecoder, native, synth

    F, L, soft = a.frames, a.frame_bits, not a.hard
    unc, rx = synth.make_frames(7, (0o113, 0o171), F, L, soft=soft, snr_db=-5.0, p=0.0559, seed=314)
    x = torch.from_numpy(rx.reshape(F, -1)).cuda()
    dec = ViterbiDecoder(ConvCode(), frame_bits=L, soft=soft)
    out = torch.empty((F, (L + 7) // 8), dtype=torch.uint8, device="cuda")
    buf = torch.zeros(8 * F, dtype=torch.int64, device="cuda")  # >= 8 u64 per wave
    lib = native.lib()
    lib.vtb_debug_set_tstamp.argtypes = [ctypes.c_void_p]
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(3):
        dec.decode_device(x, out=out, stream=s)
    torch.cuda.synchronize()
    for i in range(a.reps):
        if i == a.reps // 2:
            lib.vtb_debug_set_tstamp(ctypes.c_void_p(buf.data_ptr()))
        dec.decode_device(x, out=out, stream=s)
        if i == a.reps // 2:
            lib.vtb_debug_set_tstamp(None)
    torch.cuda.synchronize()
    b = buf.cpu().numpy().reshape(-1, 8).astype(np.int64)
    b = b[b[:, 0] != 0]
    if a.raw:
        np.save(a.raw, b)
    t0 = b[:, 0].min()
    ent, acs, tb, ex = (b[:, k] - t0 for k in range(4))
    us = 0.01  # 100 MHz realtime ticks
    clk = (b[:, 5] - b[:, 4]) / np.maximum(b[:, 3] - b[:, 0], 1) / us / 1e3  # GHz
    hw = b[:, 6]
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 31  # cu_id, sh_id
    se = (hw >> 13) & 7
    xcc = b[:, 7] & 15
    key = ((xcc * 8 + se) * 32 + cu) * 4 + simd
    uk, inv = np.unique(key, return_inverse=True)
    per_simd = np.bincount(inv)
    # the two waves of a SIMD: first-started vs second-started ACS time, and the SIMD's end
    older, younger, lone = [], [], []
    for k in range(len(uk)):
        w = np.nonzero(inv == k)[0]
        if len(w) != 2:
            continue
        w = w[np.argsort(ent[w])]
        older.append(acs[w[0]] - ent[w[0]])
        younger.append(acs[w[1]] - ent[w[1]])
        lone.append(abs(acs[w[1]] - acs[w[0]]))

    def q(v):
        return {p: round(float(np.percentile(v, p)) * us, 3) for p in (0, 10, 50, 90, 100)}

    r = {"frames": F, "frame_bits": L, "soft": soft, "waves": int(len(b)),
         "span_us": round(float(ex.max()) * us, 3),
         "entry_us": q(ent), "acs_us": q(acs - ent), "traceback_us": q(tb - acs), "copyout_us": q(ex - tb),
         "exit_us": q(ex), "clock_ghz": {p: round(float(np.percentile(clk, p)), 3) for p in (10, 50, 90)},
         "waves_per_simd": {int(k): int(v) for k, v in zip(*np.unique(per_simd, return_counts=True))},
         "simds_used": int(len(per_simd)),
         "pair_first_started_acs_us": q(np.array(older)) if older else None,
         "pair_second_started_acs_us": q(np.array(younger)) if younger else None,
         "pair_acs_end_gap_us": q(np.array(lone)) if lone else None,
         "pair_first_finishes_first": float(np.mean(np.array(older) < np.array(younger))) if older else None}
    print(json.dumps(r))
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(r, fh)


if __name__ == "__main__":
    main()
