"""Summary of tools/plant_pmc.sh (dev tool): per-wave counters of plant_step_kernel for each settings variant
of tools/plant_profile.py (7 dispatches per variant, the timed 5 averaged) and the differences that isolate the
setup (max_iter = 1), one plain iteration ((24) - (1)) / 23 and one check ((25) - (24)).
usage: python tools/plant_pmc.py <dir>"""
import collections
import csv
import glob
import sys

VARIANTS = ["default", "max_iter=1", "scaling=0,max_iter=1", "max_iter=25", "max_iter=24", "no_adapt"]
d = sys.argv[1]
per = collections.defaultdict(dict)  # dispatch -> counter -> value
for f in sorted(glob.glob(f"{d}/p*/**/*counter_collection.csv", recursive=True)):
    p = f.split("/p")[-1].split("/")[0]
    for r in csv.DictReader(open(f)):
        if "plant_step_kernel" not in r["Kernel_Name"]:
            continue
        per[(p, int(r["Dispatch_Id"]))][r["Counter_Name"]] = float(r["Counter_Value"])
byvar = collections.defaultdict(lambda: collections.defaultdict(list))
for p in sorted({k[0] for k in per}):
    ds = sorted(k for k in per if k[0] == p)
    for i, k in enumerate(ds):
        v = VARIANTS[i // 7] if i // 7 < len(VARIANTS) else f"v{i // 7}"
        if i % 7 >= 2:  # (the timed calls)
            for c, x in per[k].items():
                byvar[v][c].append(x)
avg = {v: {c: sum(x) / len(x) for c, x in cs.items()} for v, cs in byvar.items()}
keys = sorted({c for cs in avg.values() for c in cs})
print(f"{'counter (per dispatch)':24s}" + "".join(f"{v:>22s}" for v in VARIANTS if v in avg))
for c in keys:
    print(f"{c:24s}" + "".join(f"{avg[v].get(c, float('nan')):22.4g}" for v in VARIANTS if v in avg))
w = {v: avg[v].get("SQ_WAVES", 0) for v in avg}
print()
for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_WAVE_CYCLES", "SQ_ACTIVE_INST_VALU"):
    if c not in keys:
        continue
    pw = {v: avg[v][c] / w[v] for v in avg if w[v]}
    line = f"{c + ' per wave':28s} " + "  ".join(f"{v} {pw[v]:.0f}" for v in VARIANTS if v in pw)
    print(line)
    if all(k in pw for k in ("max_iter=1", "max_iter=24", "max_iter=25")):
        print(f"    setup + 1 iteration {pw['max_iter=1']:.0f}; per plain iteration {(pw['max_iter=24'] - pw['max_iter=1']) / 23:.1f}; "
              f"one check {pw['max_iter=25'] - pw['max_iter=24']:.0f}; default whole {pw.get('default', 0):.0f}")
if "GRBM_GUI_ACTIVE" in keys and "SQ_WAVE_CYCLES" in keys:
    for v in VARIANTS:
        if v in avg and avg[v].get("GRBM_GUI_ACTIVE"):
            simd = 1024 * avg[v]["GRBM_GUI_ACTIVE"] / 8
            print(f"{v:22s} waves/SIMD {4 * avg[v]['SQ_WAVE_CYCLES'] / simd:.2f}  VALU-active/wave-cycle "
                  f"{avg[v].get('SQ_ACTIVE_INST_VALU', 0) / avg[v]['SQ_WAVE_CYCLES']:.3f}")
