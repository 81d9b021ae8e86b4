"""Per-dispatch PMC summary of a tools/pmc.sh run (dev tool): python tools/pmc_phase.py gpurun_out/pmc_f32"""
import collections
import csv
import glob
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_f32"
per = collections.defaultdict(dict)
names = {}
for f in sorted(glob.glob(f"{d}/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if "admm_" not in r["Kernel_Name"]:
            continue
        key = (f, int(r["Dispatch_Id"]))
        per[key][r["Counter_Name"]] = per[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        names[key] = r["Kernel_Name"].split("<")[0].split("::")[-1]
        per[key]["_dur"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
files = sorted(set(k[0] for k in per))
for f in files:
    keys = sorted(k for k in per if k[0] == f)[-10:]
    print(f)
    for k in keys:
        c = per[k]
        line = f"  {names[k][:16]:16s} {c['_dur']:8.1f}us"
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c and "GRBM_GUI_ACTIVE" in c:
            gui = c["GRBM_GUI_ACTIVE"] / 8  # per XCD
            line += f" mfma_util={c['SQ_VALU_MFMA_BUSY_CYCLES'] / (gui * 1024):.3f} clk={gui / c['_dur'] / 1e3:.2f}GHz"
        for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if n in c and "SQ_WAVE_CYCLES" in c:
                line += f" {n[3:]}={c[n] / c['SQ_WAVE_CYCLES']:.2f}"
        for n in ("SQ_INSTS_MFMA", "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_WAVES", "FETCH_SIZE", "WRITE_SIZE"):
            if n in c:
                line += f" {n.replace('SQ_INSTS_', '')}={c[n]:.3g}"
        print(line)
