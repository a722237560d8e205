"""Average decode-kernel duration per launch from a rocprofv3 --kernel-trace --stats run
(its kernel_stats.csv), stamped with the library it was measured on, into
profiles/kernel_time.json: {workload_key: {"avg_ns", "kernel", "calls", "lib_sha16"}}.
bench.py reports it as roofline.rocprof_avg_ms beside its own event-timed kernel_avg_ms.

    python tools/kernel_time_summary.py <dir holding *kernel_stats.csv> <workload_key>
"""
import csv
import glob
import hashlib
import json
import os
import sys

repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DECODERS = ("k7_lds_kernel", "k9_kernel", "lds_path")


def main():
    root, key = sys.argv[1], sys.argv[2]
    paths = glob.glob(os.path.join(root, "**", "*kernel_stats*.csv"), recursive=True)
    if not paths:
        raise SystemExit(f"no kernel_stats.csv under {root}")
    best = None
    for r in csv.DictReader(open(paths[0])):
        if any(k in r["Name"] for k in DECODERS):
            calls, avg = int(r["Calls"]), float(r["AverageNs"])
            if best is None or calls * avg > best[1] * best[2]:  # the kernel with most GPU time
                best = (r["Name"], calls, avg)
    if best is None:
        raise SystemExit("no decode kernel in the stats")
    with open(os.path.join(repo, "convolutionalencdec_amd", "lib", "libviterbi_amd.so"), "rb") as fh:
        sha = hashlib.sha256(fh.read()).hexdigest()[:16]
    path = os.path.join(repo, "profiles", "kernel_time.json")
    data = json.load(open(path)) if os.path.exists(path) else {}
    data[key] = {"avg_ns": round(best[2], 1), "kernel": best[0], "calls": best[1], "lib_sha16": sha,
                 "source": os.path.relpath(paths[0], repo)}
    json.dump(data, open(path, "w"), indent=1, sort_keys=True)
    print(key, data[key])


if __name__ == "__main__":
    main()
