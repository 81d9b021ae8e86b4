"""Per-plant setup timing (dev tool): BatchSolver.setup of B perturbed config-3 plants, wave vs
workgroup setup kernel (MPCQ_SETUP=ref).  Wall time includes the host->device copies."""
import os
import sys
import time

import numpy as np
import torch  # noqa: F401  (share torch's HIP runtime)

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import solvempc_amd as sm  # noqa: E402
from solvempc_amd import mpc, workload  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
N = 20
plant = workload.reference_plant()
rng = np.random.default_rng(0)
Ad = plant["Ad"][None] * (1 + 0.02 * rng.normal(size=(B, 4, 4)))
Bd = plant["Bd"][None] * (1 + 0.02 * rng.normal(size=(B, 4)))
t0 = time.perf_counter()
ops = mpc.condense({"Ad": Ad, "Bd": Bd, "Cd": np.tile(plant["Cd"], (B, 1)), "K": np.tile(plant["K"], (B, 1)),
                    "Q": np.full(B, plant["Q"]), "R": np.full(B, plant["R"]), "RD": np.full(B, plant["RD"])}, N)
print(f"condense {B} plants: {time.perf_counter() - t0:.3f} s", flush=True)
l = np.full((B, 2 * N), -np.finfo(np.float64).max)
u0 = np.full((B, 2 * N), 255.0)
for mode in sys.argv[2:] or ["wave", "ref"]:
    os.environ["MPCQ_SETUP"] = mode
    s = sm.BatchSolver(N, 2 * N, B, n_plants=B)
    for rep in range(2):
        t0 = time.perf_counter()
        s.setup(ops["P"], np.zeros((B, N)), ops["A"], l, u0)
        print(f"setup[{mode}] {B} plants rep {rep}: {time.perf_counter() - t0:.3f} s", flush=True)
    s.close()
