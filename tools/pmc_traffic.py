"""HBM traffic per solve from a tools/pmc.sh FETCH_SIZE / WRITE_SIZE run (dev tool).

Sums the counters over the ADMM kernels' dispatches of the bench's solves and divides by the number
of solves (warmup + steps).  FETCH_SIZE is doubled (MI355X_MICROARCH.md HBM: on gfx950 it reports
half the bytes of wide coalesced reads); WRITE_SIZE is taken as is.  Writes
profiles/pmc_traffic_<dtype>.json for bench.py's roofline.traffic."""
import csv
import glob
import json
import sys

d, dtype, solves, batch, horizon = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
tot = {}
for f in glob.glob(f"{d}/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "admm_" not in r["Kernel_Name"]:
            continue
        tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
fetch = tot.get("FETCH_SIZE", 0.0) * 1024 / solves
write = tot.get("WRITE_SIZE", 0.0) * 1024 / solves
rec = {"dtype": dtype, "batch": batch, "horizon": horizon, "solves": solves,
       "fetch_size_bytes_raw": fetch, "write_size_bytes": write,
       "bytes_per_solve": 2 * fetch + write,
       "note": "admm_* kernels only; FETCH_SIZE x2 per the gfx950 calibration (wide coalesced reads), "
               "WRITE_SIZE as reported; rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes"}
print(json.dumps(rec, indent=1))
json.dump(rec, open(f"profiles/pmc_traffic_{dtype}.json", "w"), indent=1)
