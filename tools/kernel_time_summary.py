"""Average decode-kernel duration per launch from a rocprofv3 --kernel-trace --stats run of
bench.py, stamped with the library it was measured on, into profiles/kernel_time.json:
{workload_key: {"avg_ns", "kernel", "calls", "lib_sha16", ...}}.  bench.py reports it as
roofline.rocprof_avg_ms beside its own event-timed kernel_avg_ms.

With the run's kernel trace (*kernel_trace*.csv) the average is taken over the timed region's
dispatches only.  bench.py launches W warm-up steps back to back, synchronises, then the K timed
ones back to back, then its untimed passes (the back-to-back average pass, a pass with an event
after every launch, the host-buffer path).  The trace is cut into bursts at idle gaps
(> 10 us between one dispatch's end and the next one's start); the timed region is the first K
dispatches of the first burst of at least K that follows the warm-up burst (at least W).  The
chosen dispatch indices are recorded in the entry.  Without a trace: the stats file's average
over every dispatch.

The library stamp is the sha written next to the profile by the run that profiled it
(<dir>/lib_sha16.txt, tools/gpu_round.sh prof), not the library present when this script runs;
the directory must hold exactly one stats file and at most one trace.

    python tools/kernel_time_summary.py <dir> <workload_key> [--warmup W --steps K]
"""
import argparse
import csv
import glob
import json
import os
import statistics

repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DECODERS = ("k7_lds_kernel", "k9_kernel", "k9s_kernel", "lds_path")


def timed_window(span, warmup, steps, gap_ns=10_000):
    """Index of the timed region's first dispatch in a start-sorted [(start, end)] trace."""
    bursts, b0 = [], 0
    for i in range(1, len(span) + 1):
        if i == len(span) or span[i][0] - span[i - 1][1] > gap_ns:
            bursts.append((b0, i - b0))
            b0 = i
    seen_warm = warmup == 0
    for lo, n in bursts:
        if seen_warm and n >= steps:
            return lo
        if n >= warmup:
            seen_warm = True
    raise SystemExit(f"no burst of {steps} dispatches after a warm-up burst of {warmup}: bursts {bursts[:12]}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("key")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    stats = glob.glob(os.path.join(a.root, "**", "*kernel_stats*.csv"), recursive=True)
    if len(stats) != 1:
        raise SystemExit(f"{len(stats)} kernel stats csv under {a.root}: need exactly one run")
    sha_file = os.path.join(a.root, "lib_sha16.txt")
    if not os.path.exists(sha_file):
        raise SystemExit(f"{sha_file} missing: the profiled run's library stamp")
    lib_sha16 = open(sha_file).read().split()[-1].strip()
    best = None
    for r in csv.DictReader(open(stats[0])):
        if any(k in r["Name"] for k in DECODERS):
            calls, avg = int(r["Calls"]), float(r["AverageNs"])
            if best is None or calls * avg > best[1] * best[2]:  # the kernel with most GPU time
                best = (r["Name"], calls, avg)
    if best is None:
        raise SystemExit("no decode kernel in the stats")
    ent = {"kernel": best[0], "calls": best[1], "avg_ns_all_dispatches": round(best[2], 1)}
    traces = glob.glob(os.path.join(a.root, "**", "*kernel_trace*.csv"), recursive=True)
    if len(traces) > 1:
        raise SystemExit(f"{len(traces)} kernel traces under {a.root}: need one run")
    if traces:
        rows = [r for r in csv.DictReader(open(traces[0])) if r["Kernel_Name"] == best[0]]
        rows.sort(key=lambda r: int(r["Start_Timestamp"]))
        span = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
        lo = timed_window(span, a.warmup, a.steps)
        d = [e - s for s, e in span[lo:lo + a.steps]]
        ent.update({"avg_ns": round(statistics.mean(d), 1), "median_ns": round(statistics.median(d), 1),
                    "window": f"timed region: dispatches {lo}..{lo + a.steps - 1} of {len(span)} (0-based, "
                              "first burst of >= K after the warm-up burst)",
                    "trace": os.path.relpath(traces[0], repo)})
    else:
        ent.update({"avg_ns": round(best[2], 1), "window": "every dispatch"})
    ent["lib_sha16"] = lib_sha16
    ent["stats"] = os.path.relpath(stats[0], repo)
    path = os.path.join(repo, "profiles", "kernel_time.json")
    data = json.load(open(path)) if os.path.exists(path) else {}
    data[a.key] = ent
    json.dump(data, open(path, "w"), indent=1, sort_keys=True)
    print(a.key, {k: v for k, v in ent.items() if k != "kernel"})


if __name__ == "__main__":
    main()
