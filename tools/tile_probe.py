"""Latency/throughput probes of the tile kernel (dev tool, run on the GPU box).

Times fixed-iteration solves (eps = 0 => every QP runs exactly max_iter iterations) at several batch
sizes and check intervals, so the per-iteration and per-check costs can be separated."""
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import solvempc_amd as sm  # noqa: E402
from solvempc_amd import mpc, workload  # noqa: E402


def main():
    dtype = sys.argv[1] if len(sys.argv) > 1 else "f32"
    plant = workload.reference_plant()
    N = 20
    ops = mpc.condense({k: (plant[k][None] if k in ("Ad", "Bd", "Cd", "K") else [plant[k]])
                        for k in ("Ad", "Bd", "Cd", "K", "Q", "R", "RD")}, N)
    ops = {k: v[0] for k, v in ops.items()}
    l = np.full(2 * N, -np.finfo(np.float64).max)
    out = []
    for B in (16, 4096, 65536):
        X, U = workload.mpc_states(1, 0, B)
        q = X @ ops["Fx"].T + U[:, None] * ops["Fu"]
        u = ops["W0"] + X @ ops["Sbar"].T + U[:, None] * ops["Ku"]
        for ct, it in ((1, 100), (25, 100), (100, 100), (200, 200)):
            st = sm.default_settings(eps_abs=0.0, eps_rel=1e-30, max_iter=it, check_termination=ct,
                                     adaptive_rho=0)
            s = sm.BatchSolver(N, 2 * N, B, dtype=dtype, settings=st)
            s.setup(ops["P"], np.zeros(N), ops["A"], l, ops["W0"])
            s.update_lin_cost(q)
            s.update_upper_bound(u)
            ts = []
            for rep in range(4):
                s.reset_state()
                s.info()
                t0 = time.perf_counter()
                s.solve()
                s.info()
                ts.append(time.perf_counter() - t0)
            rec = {"B": B, "ct": ct, "iters": it, "ms": 1e3 * min(ts[1:])}
            out.append(rec)
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
