"""HBM traffic per launch from the two rocprofv3 --pmc passes of tools/gpu_check.sh pmc
(FETCH_SIZE and WRITE_SIZE, KiB per dispatch, summed over the XCDs by rocprofv3).

Writes profiles/pmc_traffic.json: {workload_key: bytes_per_launch}, read by bench.py for
roofline.traffic, plus profiles/<round>/pmc_traffic_detail.json with the raw numbers.
FETCH_SIZE/WRITE_SIZE count the L2's memory-side requests (Infinity-Cache hits included);
MI355X_MICROARCH.md: gfx950 FETCH_SIZE counts 128-B read requests as 64 B, i.e. half the
bytes of a coalesced streaming read.  This kernel's input loads are coalesced 2-byte loads
and the raw FETCH_SIZE came out at 0.517x the input bytes (4,467,188 of 8,437,760 at
K7_soft_F4096_L1024), the same halving, so the fetch figure is doubled; WRITE_SIZE matched
the output bytes exactly (524,288) and is used as is.
"""
import csv
import json
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"  # holds pmc_fetch/, pmc_write/, pmc_valu/
rnd = sys.argv[2] if len(sys.argv) > 2 else "r01"
key = sys.argv[3] if len(sys.argv) > 3 else "K7_soft_F4096_L1024"
repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# every entry is stamped with the library it was measured on (bench.py reports null for counters
# of any other binary): the sha the profiling run wrote beside its passes (tools/pmc_passes.sh,
# <root>/lib_sha16.txt), not the library present when this script runs
_sha = os.path.join(root, "lib_sha16.txt")
if not os.path.exists(_sha):
    raise SystemExit(f"{_sha} missing: the profiled run's library stamp")
LIB_SHA16 = open(_sha).read().split()[-1].strip()


def mean_counter(d, name):
    """Counter per decode launch: the mean over dispatches of each decoder kernel, summed over
    the kernels (a launch may be two dispatches: the persistent split kernel and its list
    kernel)."""
    per = {}
    for r in csv.DictReader(open(os.path.join(root, d, "run_counter_collection.csv"))):
        # the decoder's dispatches only (not the device frame generator's or runtime copies)
        if r["Counter_Name"] == name and any(k in r["Kernel_Name"] for k in ("k7_lds_kernel", "k9_kernel", "k9s_kernel", "lds_path")):
            per.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    return sum(sum(v) / len(v) for v in per.values()), max(len(v) for v in per.values())


fetch_kib, nf = mean_counter("pmc_fetch", "FETCH_SIZE")
write_kib, nw = mean_counter("pmc_write", "WRITE_SIZE")
tag = key  # detail files per workload
FETCH_CORRECTION = 2.0
total = (FETCH_CORRECTION * fetch_kib + write_kib) * 1024.0
os.makedirs(os.path.join(repo, "profiles", rnd), exist_ok=True)
with open(os.path.join(repo, "profiles", rnd, f"pmc_traffic_detail_{tag}.json"), "w") as fh:
    json.dump({"workload": key, "lib_sha16": LIB_SHA16, "fetch_kib_per_dispatch_raw": fetch_kib, "fetch_correction": FETCH_CORRECTION,
               "write_kib_per_dispatch": write_kib,
               "dispatches": [nf, nw], "bytes_per_launch": total}, fh, indent=1)
path = os.path.join(repo, "profiles", "pmc_traffic.json")
data = {}
if os.path.exists(path):
    data = json.load(open(path))
data[key] = {"bytes_per_launch": round(total), "lib_sha16": LIB_SHA16}
json.dump(data, open(path, "w"), indent=1, sort_keys=True)
print(key, "fetch KiB", fetch_kib, "write KiB", write_kib, "bytes/launch", total)

# VALU issue pass (tools/gpu_check.sh pmc, third run): wave-level VALU instructions per launch,
# for bench.py's roofline.secondary.  SQ counters are summed over the XCDs by rocprofv3;
# GRBM_GUI_ACTIVE is summed over the 8 XCDs (MI355X_MICROARCH.md, DVFS give-back).
if os.path.exists(os.path.join(root, "pmc_valu", "run_counter_collection.csv")):
    names = ("SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES",
             "SQ_ACTIVE_INST_VALU", "GRBM_GUI_ACTIVE")
    v = {n: mean_counter("pmc_valu", n)[0] for n in names}
    kt = os.path.join(root, "pmc_valu", "run_kernel_trace.csv")
    durs = {}
    for r in csv.DictReader(open(kt)):
        if any(k in r["Kernel_Name"] for k in ("k7_lds_kernel", "k9_kernel", "k9s_kernel", "lds_path")):
            durs.setdefault(r["Kernel_Name"], []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    dur_ns = sum(sum(v) / len(v) for v in durs.values())  # per launch (all its dispatches)
    v["kernel_ns_profiled"] = dur_ns
    v["effective_clock_ghz"] = v["GRBM_GUI_ACTIVE"] / 8.0 / dur_ns
    with open(os.path.join(repo, "profiles", rnd, f"pmc_valu_detail_{tag}.json"), "w") as fh:
        json.dump({"workload": key, **v}, fh, indent=1)
    vpath = os.path.join(repo, "profiles", "pmc_valu.json")
    vd = json.load(open(vpath)) if os.path.exists(vpath) else {}
    # (effective_clock_ghz reads high on dispatches shorter than ~0.3 ms: kept in the detail file only)
    vd[key] = {"valu_wave_insts_per_launch": round(v["SQ_INSTS_VALU"]), "waves_per_launch": round(v["SQ_WAVES"]),
               "lib_sha16": LIB_SHA16}
    json.dump(vd, open(vpath, "w"), indent=1, sort_keys=True)
    print(key, "VALU insts/launch", v["SQ_INSTS_VALU"], "waves", v["SQ_WAVES"], "clock GHz", v["effective_clock_ghz"])
