"""MFMA utilisation per kernel from a tools/pmc.sh run (dev tool): python tools/pmc_mfma.py <dir> <out.json>
[kernel_substr ...].  util = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs), summed over
the kernel's dispatches (MI355X_MICROARCH.md: the busy counter counts the cycles each MFMA holds its SIMD;
GRBM_GUI_ACTIVE is summed over the 8 XCDs).  Also the MFMA share of the vector instructions and, where the
MOPS counters were collected, the MFMA FLOPs (MOPS x 512)."""
import collections
import csv
import glob
import json
import sys

d, out = sys.argv[1], sys.argv[2]
pats = sys.argv[3:] or ["admm_tile_kernel"]
tot = {p: collections.defaultdict(float) for p in pats}
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        for p in pats:
            if p in r["Kernel_Name"]:
                tot[p][r["Counter_Name"] + "@" + f] += float(r["Counter_Value"])
rec = {}
for p in pats:
    # counters of one pass (file) are from the same dispatches: pair BUSY with that pass's GRBM_GUI_ACTIVE
    by_file = collections.defaultdict(dict)
    for k, v in tot[p].items():
        name, f = k.split("@", 1)
        by_file[f][name] = v
    r = {}
    for f, c in by_file.items():
        g = c.get("GRBM_GUI_ACTIVE")
        if g and "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            r["mfma_util"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * g / 8)
            r["mfma_busy_cycles"] = c["SQ_VALU_MFMA_BUSY_CYCLES"]
            r["active_cycles_per_xcd"] = g / 8
        if "SQ_INSTS_MFMA" in c and "SQ_INSTS_VALU" in c:
            r["mfma_insts"] = c["SQ_INSTS_MFMA"]
            r["valu_insts"] = c["SQ_INSTS_VALU"]
        for k in ("SQ_INSTS_VALU_MFMA_MOPS_F32", "SQ_INSTS_VALU_MFMA_MOPS_F64"):
            if k in c:
                r[k] = c[k]
                r[k.replace("SQ_INSTS_VALU_MFMA_MOPS", "mfma_flops")] = c[k] * 512
    rec[p] = r
print(json.dumps(rec, indent=1))
json.dump(rec, open(out, "w"), indent=1)
