"""Per-solve kernel sequence (durations, gaps) of each trace under gpurun_out/ab (dev tool)."""
import csv
import glob
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 6
for tr in sorted(glob.glob(f"{d}/tr_*/**/*kernel_trace.csv", recursive=True)):
    rows = sorted(csv.DictReader(open(tr)), key=lambda r: int(r['Start_Timestamp']))
    name = tr.split('/tr_')[1].split('/')[0]
    ad = [r for r in rows if 'admm' in r['Kernel_Name']]
    out = []
    for r in ad[-n:]:
        k = r['Kernel_Name']
        kind = 'wave' if 'wave' in k else ('tile' if 'tile' in k else 'lane')
        out.append(f"{kind}:{(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3:.1f}us(v{r['VGPR_Count']})")
    print(f"{name:12s}", " ".join(out))
