"""Per-stage cycle profile of the per-plant setup kernel (dev tool; MPCQ_SETUP_PROF hook)."""
import os
import sys

import numpy as np
import torch  # noqa: F401

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import solvempc_amd as sm  # noqa: E402
from solvempc_amd import mpc, workload  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
N = 20
plant = workload.reference_plant()
Ad, Bd = workload.randomized_plants(plant, 2, 0, B)
ops = mpc.condense({"Ad": Ad, "Bd": Bd, "Cd": np.tile(plant["Cd"], (B, 1)), "K": np.tile(plant["K"], (B, 1)),
                    "Q": np.full(B, plant["Q"]), "R": np.full(B, plant["R"]), "RD": np.full(B, plant["RD"])}, N)
out = os.path.abspath("gpurun_out/setup_prof.bin")
os.makedirs(os.path.dirname(out), exist_ok=True)
os.environ["MPCQ_SETUP_PROF"] = out
s = sm.BatchSolver(N, 2 * N, B, n_plants=B)
s.setup(ops["P"], np.zeros((B, N)), ops["A"], np.full((B, 2 * N), -1.7e308), np.full((B, 2 * N), 255.0))
h = np.fromfile(out, dtype=np.int64).reshape(B, 16)
names = ["load", "ruiz", "types", "Pt/G", "chol", "C", "jacobi", "outputs"]
d = np.diff(h[:, :9], axis=1)
tot = h[:, 8] - h[:, 0]
print(f"B={B} total cycles/plant: mean {tot.mean():.0f}  median {np.median(tot):.0f}")
for k, nm in enumerate(names):
    print(f"  {nm:8s} {d[:, k].mean():10.0f}  {100 * d[:, k].mean() / tot.mean():5.1f}%")
print("jacobi sweeps: mean", h[:, 15].mean(), "max", h[:, 15].max())
