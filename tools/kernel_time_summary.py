"""Average decode-kernel duration per launch from a rocprofv3 --kernel-trace --stats run of
bench.py, stamped with the library it was measured on, into profiles/kernel_time.json:
{workload_key: {"avg_ns", "kernel", "calls", "lib_sha16", ...}}.  bench.py reports it as
roofline.rocprof_avg_ms beside its own event-timed kernel_avg_ms.

With the run's kernel trace (*kernel_trace*.csv) the average is taken over the timed region's
dispatches only (bench.py launches W warm-up steps, then the K timed ones, then its untimed
passes: the back-to-back average pass, a pass with an event after every launch, and the
host-buffer path, whose launches follow idle gaps and run slower); without it, the stats
file's average over every dispatch.

    python tools/kernel_time_summary.py <dir> <workload_key> [--warmup W --steps K]
"""
import argparse
import csv
import glob
import hashlib
import json
import os
import statistics

repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DECODERS = ("k7_lds_kernel", "k9_kernel", "lds_path")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("key")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    stats = glob.glob(os.path.join(a.root, "**", "*kernel_stats*.csv"), recursive=True)
    if not stats:
        raise SystemExit(f"no kernel stats csv under {a.root}")
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
    if traces:
        rows = [r for r in csv.DictReader(open(traces[0])) if r["Kernel_Name"] == best[0]]
        rows.sort(key=lambda r: int(r["Start_Timestamp"]))
        d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows][a.warmup:a.warmup + a.steps]
        ent.update({"avg_ns": round(statistics.mean(d), 1), "median_ns": round(statistics.median(d), 1),
                    "window": f"timed region: dispatches {a.warmup}..{a.warmup + a.steps - 1}",
                    "trace": os.path.relpath(traces[0], repo)})
    else:
        ent.update({"avg_ns": round(best[2], 1), "window": "every dispatch"})
    with open(os.path.join(repo, "convolutionalencdec_amd", "lib", "libviterbi_amd.so"), "rb") as fh:
        ent["lib_sha16"] = hashlib.sha256(fh.read()).hexdigest()[:16]
    ent["stats"] = os.path.relpath(stats[0], repo)
    path = os.path.join(repo, "profiles", "kernel_time.json")
    data = json.load(open(path)) if os.path.exists(path) else {}
    data[a.key] = ent
    json.dump(data, open(path, "w"), indent=1, sort_keys=True)
    print(a.key, {k: v for k, v in ent.items() if k != "kernel"})


if __name__ == "__main__":
    main()
