"""Diagnostic (GPU): how the fp32 device path's iteration schedule diverges from the fp64 oracle.
Prints, per kernel path, the fraction of QPs on another schedule, their oracle decision margins and
the worst |x - x_oracle| on the applied move and the whole vector."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401,E402
import oracle  # noqa: E402
import solvempc_amd as sm  # noqa: E402
from solvempc_amd import workload  # noqa: E402

N, B = 20, int(os.environ.get("DIAG_B", "4096"))
plant = workload.reference_plant()
ops = oracle.condense(plant, N)
X, U = workload.mpc_states(1, 0, B)
q, u = oracle.gradient(ops, X, U), oracle.upper_bound(ops, X, U)
l = np.full(2 * N, -np.finfo(np.float64).max)
u0 = oracle.upper_bound(ops, np.zeros(4), 0.0)
xr, sr, ir, rr, mg = oracle.batch_solve(ops["P"], ops["A"], np.zeros(N), l, u0, q, u, margins=True)
for kern in ("tile", "wave"):
    os.environ["MPCQ_KERNEL"] = kern
    for dt in ("f32", "f64"):
        s = sm.BatchSolver(N, 2 * N, B, dtype=dt)
        s.setup(ops["P"], np.zeros(N), ops["A"], l, u0)
        s.update_lin_cost(q)
        s.update_upper_bound(u)
        s.solve()
        x = s.solution()
        st, it, rho = s.info()
        d = it != ir
        e0 = np.abs(x[:, 0] - xr[:, 0])
        ev = np.abs(x - xr).max(axis=1) / np.maximum(1, np.abs(xr).max(axis=1))
        print(f"{kern} {dt}: diverge {d.mean():.4%} ({d.sum()}); margin of diverging: "
              f"{np.sort(mg[d])[:8]} max {mg[d].max() if d.any() else 0:.3e}; "
              f"|dx0| all {e0.max():.2e} same {e0[~d].max():.2e} div {e0[d].max() if d.any() else 0:.2e}; "
              f"rel vec same {ev[~d].max():.2e} div {ev[d].max() if d.any() else 0:.2e}; "
              f"rho rel {np.abs(rho[~d] / rr[~d] - 1).max():.2e}", flush=True)
        for thr in (1e-3, 3e-3, 1e-2, 3e-2, 1e-1):
            print(f"   margin<{thr:g}: {(mg < thr).mean():.4%}  diverging with margin>={thr:g}: {(d & (mg >= thr)).sum()}")
        s.close()
