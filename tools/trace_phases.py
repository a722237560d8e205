"""Summarise a rocprofv3 kernel trace of `bench.py` by phase (measurement only).

    python tools/trace_phases.py <run_kernel_trace.csv> [--warmup W] [--steps K]

The bench issues, on one stream, one launch from ViterbiDecoder.bind (validation), W warm-up launches, the K timed launches (back to back,
nothing between them), K launches with an event after each (the untimed per-launch pass) and
then the host-path launches.  Prints per phase: count, mean / min / median / max duration (us)
and the mean gap before each launch, for the decoder kernel (the dispatches whose name holds
`k7_lds_kernel`, `k9_kernel`, `k9s_kernel` or `lds_path`)."""
import argparse
import csv
import json

import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    rows = [r for r in csv.DictReader(open(a.trace))
            if any(k in r["Kernel_Name"] for k in ("k7_lds_kernel", "k9_kernel", "k9s_kernel", "lds_path"))]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    st = np.array([int(r["Start_Timestamp"]) for r in rows], np.int64)
    en = np.array([int(r["End_Timestamp"]) for r in rows], np.int64)
    dur = (en - st) / 1e3
    gap = np.r_[np.nan, (st[1:] - en[:-1]) / 1e3]
    W, K = a.warmup + 1, a.steps  # (+1: the bind launch)
    phases = {"bind_and_warmup": (0, W), "timed": (W, W + K), "per_launch_pass": (W + K, W + 2 * K),
              "host_path": (W + 2 * K, len(rows))}
    out = {"kernel": rows[0]["Kernel_Name"][:120] if rows else None}
    for name, (lo, hi) in phases.items():
        d, g = dur[lo:hi], gap[lo:hi]
        if d.size == 0:
            continue
        out[name] = {"n": int(d.size), "mean_us": round(float(d.mean()), 3), "min_us": round(float(d.min()), 3),
                     "median_us": round(float(np.median(d)), 3), "max_us": round(float(d.max()), 3),
                     "mean_gap_between_us": round(float(np.nanmean(g[1:]) if g.size > 1 else float("nan")), 3)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
