"""HBM traffic per launch of a bench workload's dominant kernel from a tools/pmc.sh FETCH_SIZE / WRITE_SIZE
run (dev tool; tools/gpu.sh step pmc:<workload>,<dtype>).

Sums each counter over the dispatches of every kernel whose name contains one of the given substrings,
divides by the number of bench steps the run made (warmup + steps), and writes
profiles/pmc_traffic_<name>.json for bench.py's roofline.traffic.  FETCH_SIZE is doubled (MI355X_MICROARCH.md
HBM: on gfx950 it reports half the bytes of wide coalesced reads); WRITE_SIZE is taken as reported (its
calibration on the finalize's store shapes: tools/calib/write_calib.hip, profiles/r05e_calib_write.csv).
usage: python tools/pmc_traffic.py <pmc dir> <name> <steps> <batch> <horizon> <kernel substring>[,<substring>..]"""
import csv
import glob
import json
import sys

d, name, steps, batch, horizon = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
kernels = (sys.argv[6] if len(sys.argv) > 6 else "admm_").split(",")
tot, per_kernel = {}, {}
for f in glob.glob(f"{d}/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = next((k for k in kernels if k in r["Kernel_Name"]), None)
        if k is None:
            continue
        v = float(r["Counter_Value"]) * 1024  # (KB)
        tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + v
        pk = per_kernel.setdefault(k, {})
        pk[r["Counter_Name"]] = pk.get(r["Counter_Name"], 0.0) + v
fetch = tot.get("FETCH_SIZE", 0.0) / steps
write = tot.get("WRITE_SIZE", 0.0) / steps
rec = {"name": name, "batch": batch, "horizon": horizon, "steps": steps, "kernels": kernels,
       "fetch_size_bytes_raw": fetch, "write_size_bytes": write, "bytes_per_solve": 2 * fetch + write,
       "per_kernel": {k: {"fetch_x2": 2 * v.get("FETCH_SIZE", 0.0) / steps, "write": v.get("WRITE_SIZE", 0.0) / steps}
                      for k, v in per_kernel.items()},
       "note": "bytes per bench step (one solve / one controllerStep batch / one stream of control steps); "
               "FETCH_SIZE x2 per the gfx950 calibration (wide coalesced reads), WRITE_SIZE as reported; "
               "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes"}
print(json.dumps(rec, indent=1))
json.dump(rec, open(f"profiles/pmc_traffic_{name}.json", "w"), indent=1)
