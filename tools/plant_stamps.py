"""Per-wave stage stamps of plant_step_kernel (dev tool, GPU; BASELINE config 3).  Needs a debug build:
`SRC=mpcq_plant.hip DBGDIR=tools/dbg_r06p bash tools/build_dbg.sh MPCQ_PLANT_STAMPS`, run with
MPCQ_LIBRARY=tools/dbg_r06p/libmpcq.so.  Runs the bench's batch (131,072 plants, seed 2, fp64, hardest-first)
twice and prints the median shader cycles of each stage per wave (three plants) and the wave lifetimes.
Stamps: 0 entry, 1 condensing recurrences, 2 lag table + P + q (12 plant data, 13 CS scan, 14 lag table), 3 Ruiz, 4 front end, 5 first KKT inverse,
6 iteration 1, 7 iteration ct (before its check), 8 its check, 9 exit; 11 the wave's last iteration.
usage: python tools/plant_stamps.py [plants] [dtype]"""
import os
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import solvempc_amd as sm  # noqa: E402
from solvempc_amd import workload  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 131072
dtype = sys.argv[2] if len(sys.argv) > 2 else "f64"
N = 20
out = os.environ.setdefault("MPCQ_PLANT_STAMPS", "/tmp/plant_stamps.bin")
plant = workload.reference_plant()
Ad, Bd = workload.randomized_plants(plant, 2, 0, B)
X, U = workload.mpc_states(2, 0, B)
dev = torch.device("cuda:0")
t = lambda v: torch.as_tensor(np.ascontiguousarray(v, dtype=np.float64), device=dev)  # noqa: E731
pl = [t(Ad), t(Bd), t(np.tile(plant["Cd"], (B, 1))), t(np.tile(plant["K"], (B, 1))), t(np.full(B, plant["Q"])),
      t(np.full(B, plant["R"])), t(np.full(B, plant["RD"]))]
Xd, Ud = t(X), t(U)
s = sm.BatchSolver(N, 2 * N, B, n_plants=B, dtype=dtype)
for _ in range(2):
    Ud.copy_(t(U))
    s.mpc_plants_step_device(4, 10, *[x.data_ptr() for x in pl], Xd.data_ptr(), Ud.data_ptr())
torch.cuda.synchronize()
h = np.fromfile(out, dtype=np.int64).reshape(-1, 16)
h = h[h[:, 0] != 0]
print(f"waves {len(h)} ({dtype}, {B} plants)")
names = {12: "plant data loads", 1: "condensing recurrences", 13: "CS scan", 14: "lag table", 2: "P, q", 3: "Ruiz", 4: "front end", 5: "first KKT inverse",
         6: "iteration 1", 7: "iterations 2 .. ct", 8: "check at ct", 9: "rest of the solve"}
prev = h[:, 0]
for k in (12, 1, 13, 14, 2, 3, 4, 5, 6, 7, 8, 9):
    d = h[:, k] - prev
    print(f"  {k} {names[k]:24s} median {np.median(d):9.0f}  mean {d.mean():9.0f}  p90 {np.percentile(d, 90):9.0f}")
    prev = h[:, k]
life = h[:, 9] - h[:, 0]
setup = h[:, 6] - h[:, 0]
it = h[:, 11]
print(f"  wave lifetime median {np.median(life):.0f}  mean {life.mean():.0f}; setup + 1 iteration {setup.mean():.0f} "
      f"({setup.mean() / life.mean():.3f} of the mean lifetime); last iteration mean {it.mean():.1f} max {it.max()}")
per_it = (h[:, 9] - h[:, 8]) / np.maximum(1, it - 25)
print(f"  cycles per iteration after the first check (incl. checks, refactorisations): median {np.median(per_it[it > 25]):.0f}")
span = (h[:, 9].max() - h[:, 0].min())
print(f"  span of all waves {span} cycles")
