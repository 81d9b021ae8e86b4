"""Per-kernel PMC totals of every pass under a pmc output dir (dev tool): python tools/pmc_summary.py <dir> [kernel_substr]"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "admm"
tot = collections.defaultdict(float)
durs = {}
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if pat not in r["Kernel_Name"]:
            continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
        durs[(f, r["Dispatch_Id"])] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
for k in sorted(tot):
    print(f"{k:28s} {tot[k]:.4g}")
if "GRBM_GUI_ACTIVE" in tot:
    g = tot["GRBM_GUI_ACTIVE"] / 8
    print("per-XCD active cycles", f"{g:.4g}")
    simd = 1024 * g
    for k in ("SQ_VALU_MFMA_BUSY_CYCLES",):
        if k in tot:
            print(f"{k} / SIMD-cycles = {tot[k] / simd:.3f}")
    if "SQ_WAVE_CYCLES" in tot:
        w = tot["SQ_WAVE_CYCLES"]
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_BUSY_CYCLES"):
            if k in tot:
                print(f"{k} / WAVE_CYCLES = {tot[k] / w:.3f}")
        print("avg waves/SIMD =", f"{4 * w / simd:.2f}")
