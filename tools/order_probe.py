"""Probe for the hardest-first order (mpcq_order.hip): times mpc_step_device on the config-2
bench batch with the batch pre-permuted on the host (MPCQ_ORDER=0: the device keeps the given order) in index
order and in ascending |max violation of the unconstrained optimum| (exact, and binned at 2 / 4 / 8 bins per
octave with index order inside a bin), one launch (MPCQ_PHASES=0) or the default chain, and with the device's
own order (the library default).  Checks that the applied moves are bit-identical in every arrangement."""
import json
import os
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import solvempc_amd as sm  # noqa: E402
from solvempc_amd import workload  # noqa: E402

N, B = 20, 65536
dtype = sys.argv[1] if len(sys.argv) > 1 else "mixed"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
plant = workload.reference_plant()
ops = sm.mpc.condense({"Ad": plant["Ad"][None], "Bd": plant["Bd"][None], "Cd": plant["Cd"][None],
                       "K": plant["K"][None], "Q": [plant["Q"]], "R": [plant["R"]], "RD": [plant["RD"]]}, N)
ops = {k: v[0] for k, v in ops.items()}
X, U = workload.mpc_states(1, 0, B)
xref = plant["xref"]
q = X @ ops["Fx"].T + U[:, None] * ops["Fu"][None] + (ops["Fr"].sum(1) * xref)[None]
u = ops["W0"][None] + X @ ops["Sbar"].T + U[:, None] * ops["Ku"][None]
xu = -np.linalg.solve(ops["P"], q.T).T
a = np.abs((xu @ ops["A"].T - u).max(1))
orders = {"index": np.arange(B), "exact": np.argsort(a, kind="stable")}
for per in (2, 4, 8):
    orders[f"bins{per}"] = np.lexsort((np.arange(B), np.floor(per * np.log2(np.maximum(a, 1e-300)))))
l = np.full(2 * N, -np.finfo(np.float64).max)
dev = torch.device("cuda:0")
ref = None
cases = [(o, "0", "host") for o in orders] + [("index", "", "host"), ("index", "", "device")]
for oname, ph, who in cases:
    order = orders[oname]
    if who == "host":
        os.environ["MPCQ_ORDER"] = "0"
    else:
        os.environ.pop("MPCQ_ORDER", None)
    if ph:
        os.environ["MPCQ_PHASES"] = ph
    else:
        os.environ.pop("MPCQ_PHASES", None)
    s = sm.BatchSolver(N, 2 * N, B, 1, dtype, 0)
    s.setup(ops["P"], np.zeros(N), ops["A"], l, ops["W0"].copy())
    s.mpc_set_operators(ops["Fx"], ops["Fu"], ops["Fr"], ops["Sbar"], ops["Ku"], ops["W0"])
    Xd = torch.from_numpy(np.ascontiguousarray(X[order])).to(dev)
    U0 = torch.from_numpy(np.ascontiguousarray(U[order])).to(dev)
    Ud = U0.clone()
    st = torch.cuda.current_stream(dev)
    times = []
    for i in range(reps + 3):
        Ud.copy_(U0)
        s.reset_state()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        s.mpc_step_device(Xd.data_ptr(), Ud.data_ptr(), xref, st.cuda_stream)
        e1.record(st)
        torch.cuda.synchronize()
        if i >= 3:
            times.append(e0.elapsed_time(e1))
    Uo = np.empty(B)
    Uo[order] = Ud.cpu().numpy()
    if ref is None:
        ref = Uo
    print(json.dumps({"order": oname, "by": who, "phases": ph or "default", "dtype": dtype,
                      "device_ordered": s.order()[0], "ms_median": float(np.median(times)),
                      "ms_min": float(np.min(times)), "qps_M": B / float(np.median(times)) / 1e3,
                      "U_bit_identical": bool(np.array_equal(Uo, ref))}), flush=True)
    s.close()
