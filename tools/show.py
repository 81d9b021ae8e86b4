"""Summarise gpurun_out/ bench JSON lines and the last kernel trace (dev tool)."""
import csv
import glob
import json
import sys

for f in sorted(glob.glob("gpurun_out/bench_*.json")):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(f, "unreadable", e)
        continue
    r = d["roofline"]
    print(f"{f:32s} {d['dtype']} {d['value'] / 1e6:8.2f} M QP/s {d['ms_per_step']:.3f} ms/step "
          f"kernel {r['kernel_ms']:.3f} ms frac {r['frac']:.3f}")
pat = sys.argv[1] if len(sys.argv) > 1 else "admm_"
for tr in glob.glob("gpurun_out/prof*/run_kernel_trace.csv"):
    rows = [r for r in csv.DictReader(open(tr)) if pat in r["Kernel_Name"]]
    if not rows:
        continue
    last = rows[-10:]
    print(tr, [(r["Kernel_Name"].split("<")[0].split("::")[-1][:10], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) // 1000) for r in last])
