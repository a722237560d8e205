"""Write rocprofv3's kernel trace and kernel stats CSVs from a run's SQLite output
(<dir>/*_results.db, rocprofv3's default format when --output-format csv is not given): the
`kernels` view (one row per dispatch) becomes run_kernel_trace.csv (Kernel_Name,
Start_Timestamp, End_Timestamp, ...) and run_kernel_stats.csv (Name, Calls, TotalDurationNs,
AverageNs, Percentage, MinNs, MaxNs), the columns tools/kernel_time_summary.py reads.

    python tools/rocpd_to_csv.py <dir>
"""
import csv
import glob
import os
import sqlite3
import sys


def main():
    root = sys.argv[1]
    dbs = glob.glob(os.path.join(root, "*_results.db"))
    if len(dbs) != 1:
        raise SystemExit(f"{len(dbs)} result databases under {root}: need one")
    c = sqlite3.connect(dbs[0])
    rows = c.execute("select name, start, end, dispatch_id, grid_x, workgroup_x, lds_size from kernels "
                     "order by start").fetchall()
    with open(os.path.join(root, "run_kernel_trace.csv"), "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp", "Dispatch_Id", "Grid_Size", "Workgroup_Size",
                    "LDS_Block_Size"])
        for r in rows:
            w.writerow(r)
    stats = {}
    for name, s, e, *_ in rows:
        stats.setdefault(name, []).append(e - s)
    total = sum(sum(v) for v in stats.values())
    with open(os.path.join(root, "run_kernel_stats.csv"), "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for name, d in sorted(stats.items(), key=lambda kv: -sum(kv[1])):
            w.writerow([name, len(d), sum(d), sum(d) / len(d), 100.0 * sum(d) / total, min(d), max(d)])
    print(f"{len(rows)} dispatches of {len(stats)} kernels -> {root}/run_kernel_trace.csv, run_kernel_stats.csv")


if __name__ == "__main__":
    main()
