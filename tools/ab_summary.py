"""Summarise gpurun_out/ab: bench value / roofline per variant and the last solve's kernel sequence."""
import csv
import glob
import json
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab"
for f in sorted(glob.glob(f"{d}/*.json")):
    name = os.path.basename(f)[:-5]
    try:
        r = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(name, "unreadable", e)
        continue
    rf = r.get("roofline", {})
    print(f"{name:20s} value={r['value']/1e6:8.2f}M  ms/step={r['ms_per_step']:.4f} kern_ms={rf.get('kernel_ms', 0):.4f} "
          f"frac={rf.get('frac', 0):.3f}")
    tr = glob.glob(f"{d}/tr_{name}/**/*kernel_trace.csv", recursive=True)
    if tr:
        rows = list(csv.DictReader(open(tr[0])))
        ks = [(r_['Kernel_Name'].split('(')[0][-48:], (int(r_['End_Timestamp']) - int(r_['Start_Timestamp'])) / 1e3,
               r_['VGPR_Count'], r_['Accum_VGPR_Count'], r_['Grid_Size_X'], r_['LDS_Block_Size']) for r_ in rows]
        admm = [k for k in ks if 'admm' in k[0]]
        n_last = 8
        print("   last kernels:", " | ".join(f"{k[0][-22:]} {k[1]:.1f}us v{k[2]}/{k[3]} g{k[4]}" for k in admm[-n_last:]))
