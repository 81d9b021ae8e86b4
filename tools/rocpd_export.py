"""rocprofv3 SQLite output (run_results.db, the default format of this ROCm) -> the CSV summaries committed under
profiles/ (dev tool): <prefix>_kernel_stats.csv (per kernel: calls, total / average / min / max duration in ns,
percent) and <prefix>_kernel_trace.csv (per dispatch: name, start, end, duration ns, grid, workgroup, LDS,
scratch, VGPR / AGPR / SGPR counts).  usage: python tools/rocpd_export.py run_results.db <prefix>"""
import csv
import sqlite3
import sys
from collections import defaultdict

db, prefix = sys.argv[1], sys.argv[2]
c = sqlite3.connect(db)
cols = ["name", "dispatch_id", "start", "end", "duration", "grid_x", "grid_y", "grid_z", "workgroup_x", "workgroup_y",
        "workgroup_z", "lds_size", "scratch_size", "vgpr_count", "accum_vgpr_count", "sgpr_count"]
rows = c.execute(f"select {', '.join(cols)} from kernels order by start").fetchall()
with open(f"{prefix}_kernel_trace.csv", "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["Kernel_Name", "Dispatch_Id", "Start_Timestamp", "End_Timestamp", "Duration_ns", "Grid_X", "Grid_Y",
                "Grid_Z", "Workgroup_X", "Workgroup_Y", "Workgroup_Z", "LDS_Size", "Scratch_Size", "VGPR_Count",
                "Accum_VGPR_Count", "SGPR_Count"])
    w.writerows(rows)
agg = defaultdict(list)
for r in rows:
    agg[r[0]].append(r[4])
tot = sum(sum(v) for v in agg.values())
with open(f"{prefix}_kernel_stats.csv", "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "Percentage"])
    for name, d in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        w.writerow([name, len(d), sum(d), sum(d) / len(d), min(d), max(d), 100.0 * sum(d) / tot])
print(f"{len(rows)} dispatches, {len(agg)} kernels -> {prefix}_kernel_stats.csv, {prefix}_kernel_trace.csv")
