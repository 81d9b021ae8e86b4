"""Dev tool (GPU): time one cfg2 solve (65,536 shared-plant QPs, f32) under different phase lists
(MPCQ_PHASES test hook: check_termination multiples at which the tile chain re-packs; the launch after
the third runs one QP per wave).  Prints ms per solve for each setting."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import solvempc_amd as sm  # noqa: E402
from solvempc_amd import workload  # noqa: E402

N, B = 20, int(os.environ.get("B", "65536"))
dtype = os.environ.get("DTYPE", "f32")
settings = sys.argv[1:] or ["", "3,4", "3,4,5,6"]
dev = torch.device("cuda:0")
plant = workload.reference_plant()
ops = sm.mpc.condense({"Ad": plant["Ad"][None], "Bd": plant["Bd"][None], "Cd": plant["Cd"][None],
                       "K": plant["K"][None], "Q": [plant["Q"]], "R": [plant["R"]], "RD": [plant["RD"]]}, N, device=0)
ops = {k: v[0] for k, v in ops.items()}
X, U = workload.mpc_states(1, 0, B)
s = sm.BatchSolver(N, 2 * N, B, 1, dtype, 0)
s.setup(ops["P"], np.zeros(N), ops["A"], np.full(2 * N, -np.finfo(np.float64).max), ops["W0"].copy())
s.mpc_set_operators(ops["Fx"], ops["Fu"], ops["Fr"], ops["Sbar"], ops["Ku"], ops["W0"])
Xd, U0 = torch.from_numpy(X).to(dev), torch.from_numpy(U).to(dev)
Ud = U0.clone()
stream = torch.cuda.current_stream(dev)
for ph in settings:
    if ph:
        os.environ["MPCQ_PHASES"] = ph
    else:
        os.environ.pop("MPCQ_PHASES", None)
    ts = []
    for i in range(25):
        Ud.copy_(U0)
        s.reset_state()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        s.mpc_step_device(Xd.data_ptr(), Ud.data_ptr(), plant["xref"], stream.cuda_stream)
        e1.record(stream)
        torch.cuda.synchronize()
        if i >= 5:
            ts.append(e0.elapsed_time(e1))
    st, it, _ = s.info()
    print(f"phases={ph or 'default':12s} {np.mean(ts):.4f} ms (min {np.min(ts):.4f})  solved {np.mean(st == sm.SOLVED):.4f}"
          f"  iters mean {it.mean():.1f} max {it.max()}", flush=True)
