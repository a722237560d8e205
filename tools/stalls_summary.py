"""Summarise tools/pmc_stalls.sh (three SQ counter passes of the bench workload) into one JSON:
per-dispatch means over the decoder dispatches, plus the wave-cycle shares and per-wave counts.
Usage: python tools/stalls_summary.py gpurun_out/stalls <out.json> <note>"""
import collections
import csv
import glob
import json
import sys

root, out = sys.argv[1], sys.argv[2]
note = sys.argv[3] if len(sys.argv) > 3 else ""
acc = collections.defaultdict(list)
for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if any(k in r["Kernel_Name"] for k in ("k7_lds_kernel", "k9_kernel", "k9s_kernel", "lds_path")):
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {k: round(sum(v) / len(v)) for k, v in acc.items()}
wc, waves = m["SQ_WAVE_CYCLES"], m["SQ_WAVES"]
d = {k + "_share_of_wave_cycles": round(m[k] / wc, 3)
     for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS",
               "SQ_ACTIVE_INST_SCA") if k in m}
if "SQ_LDS_IDX_ACTIVE" in m:
    d["lds_bank_conflict_share_of_lds_cycles"] = round(m["SQ_LDS_BANK_CONFLICT"] / m["SQ_LDS_IDX_ACTIVE"], 3)
d["per_wave"] = {k: round(m[k] / waves, 1) for k in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM",
                                                        "SQ_LDS_BANK_CONFLICT") if k in m}
m["_derived"] = d
m["_note"] = note
json.dump(m, open(out, "w"), indent=1)
print(json.dumps(d, indent=1))
