"""Latency/throughput probes of the shared-plant ADMM kernels (dev tool, run on the GPU box).

Fixed-iteration solves (eps = 0, adaptive rho off: every QP runs exactly `iters` iterations, one
launch: MPCQ_PHASES=0) timed with HIP events on the launch stream, at several batch sizes, so that
T(B, iters) = fixed(B) + iters * per_iter(B) separates launch/prologue cost from the loop."""
import json
import os
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import solvempc_amd as sm  # noqa: E402
from solvempc_amd import mpc, workload  # noqa: E402


def main():
    import torch

    os.environ.setdefault("MPCQ_PHASES", "0")
    dtype = sys.argv[1] if len(sys.argv) > 1 else "f32"
    batches = [int(b) for b in (sys.argv[2].split(",") if len(sys.argv) > 2 else (16, 16384, 49152, 65536))]
    iters_list = [int(i) for i in (sys.argv[3].split(",") if len(sys.argv) > 3 else (25, 75, 125))]
    plant = workload.reference_plant()
    N = 20
    ops = mpc.condense({k: (plant[k][None] if k in ("Ad", "Bd", "Cd", "K") else [plant[k]])
                        for k in ("Ad", "Bd", "Cd", "K", "Q", "R", "RD")}, N)
    ops = {k: v[0] for k, v in ops.items()}
    l = np.full(2 * N, -np.finfo(np.float64).max)
    stream = torch.cuda.current_stream()
    for B in batches:
        X, U = workload.mpc_states(1, 0, B)
        q = X @ ops["Fx"].T + U[:, None] * ops["Fu"]
        u = ops["W0"] + X @ ops["Sbar"].T + U[:, None] * ops["Ku"]
        res = []
        for it in iters_list:
            st = sm.default_settings(eps_abs=0.0, eps_rel=1e-30, max_iter=it, adaptive_rho=0)
            s = sm.BatchSolver(N, 2 * N, B, dtype=dtype, settings=st)
            s.setup(ops["P"], np.zeros(N), ops["A"], l, ops["W0"])
            s.update_lin_cost(q)
            s.update_upper_bound(u)
            ts = []
            for rep in range(5):
                s.reset_state()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                s.solve(stream.cuda_stream)
                e1.record(stream)
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3)
            res.append((it, min(ts[1:])))
            s.close()
        its = np.array([r[0] for r in res], float)
        us = np.array([r[1] for r in res])
        slope, icpt = np.polyfit(its, us, 1) if len(its) > 1 else (us[0] / its[0], 0.0)
        rec = {"B": B, "dtype": dtype, "us": {int(a): round(b, 2) for a, b in res}, "us_per_iter": round(slope, 3),
               "fixed_us": round(icpt, 2), "kernel": os.environ.get("MPCQ_KERNEL", "default")}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
