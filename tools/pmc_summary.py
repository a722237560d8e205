"""Summarise rocprofv3 counter-collection CSVs (tools/pmc_sq.sh output): per-dispatch means
of every counter for the decoder kernels, and per-wave / per-step derived numbers."""
import collections
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1056
acc = collections.defaultdict(list)
for f in sorted(glob.glob(f"{root}/pmc_sq*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if "kernel" not in r["Kernel_Name"]:
            continue
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {k: sum(v) / len(v) for k, v in acc.items()}
waves = m.get("SQ_WAVES", 1)
for k in sorted(m):
    print(f"{k:28s} {m[k]:16.1f}   per wave {m[k] / waves:12.2f}   per wave-step {m[k] / waves / steps:8.3f}")
if "SQ_WAVE_CYCLES" in m:
    wc = m["SQ_WAVE_CYCLES"]
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
        if k in m:
            print(f"{k} / SQ_WAVE_CYCLES = {m[k] / wc:.3f}")
