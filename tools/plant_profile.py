"""Dev tool (GPU): time the one-pass per-plant kernel (mpcq_mpc_plants_step_device) on the config-3
batch under settings that isolate its stages: default; max_iter = 1 (condense + setup + one
iteration); scaling = 0 (no Ruiz).  Prints ms per call."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import solvempc_amd as sm  # noqa: E402
from solvempc_amd import workload  # noqa: E402

N, B = 20, int(os.environ.get("B", "131072"))
plant = workload.reference_plant()
Ad, Bd = workload.randomized_plants(plant, 2, 0, B)
X, U = workload.mpc_states(2, 0, B)
dev = torch.device("cuda:0")
t = lambda v: torch.as_tensor(np.ascontiguousarray(v, dtype=np.float64), device=dev)  # noqa: E731
pl = [t(Ad), t(Bd), t(np.tile(plant["Cd"], (B, 1))), t(np.tile(plant["K"], (B, 1))), t(np.full(B, plant["Q"])),
      t(np.full(B, plant["R"])), t(np.full(B, plant["RD"]))]
Xd, U0 = t(X), t(U)
for dtype in os.environ.get("DTYPES", "f32,f64").split(","):
    for name, over in (("default", {}), ("max_iter=1", dict(max_iter=1)), ("scaling=0,max_iter=1", dict(scaling=0, max_iter=1)),
                       ("max_iter=25", dict(max_iter=25)), ("max_iter=24", dict(max_iter=24)),
                       ("no_adapt", dict(adaptive_rho=0))):
        s = sm.BatchSolver(N, 2 * N, B, n_plants=B, dtype=dtype, settings=sm.default_settings(**over))
        Ud = U0.clone()
        for _ in range(2):
            s.mpc_plants_step_device(4, 10, *[x.data_ptr() for x in pl], Xd.data_ptr(), Ud.data_ptr())
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            s.mpc_plants_step_device(4, 10, *[x.data_ptr() for x in pl], Xd.data_ptr(), Ud.data_ptr())
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / 5 * 1e3
        st, it, _ = s.info()
        print(f"{dtype} {name:24s} {ms:8.3f} ms  iters mean {it.mean():.1f}", flush=True)
        s.close()
