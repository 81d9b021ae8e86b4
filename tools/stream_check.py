"""Closed-loop sanity of the receding-horizon stream (dev tool, GPU box): max |X|, |U| and the status
mix every 50 control steps, f32 vs f64, for the reference controller on its own plant model."""
import sys

import numpy as np
import torch

sys.path.insert(0, '.')
import solvempc_amd as sm  # noqa: E402
from solvempc_amd import mpc, workload  # noqa: E402

plant = workload.reference_plant()
N, B = 20, int(sys.argv[1]) if len(sys.argv) > 1 else 4096
ops = mpc.condense({k: (plant[k][None] if k in ("Ad", "Bd", "Cd", "K") else [plant[k]])
                    for k in ("Ad", "Bd", "Cd", "K", "Q", "R", "RD")}, N)
ops = {k: v[0] for k, v in ops.items()}
for dt in ("f64", "f32"):
    X, U = workload.mpc_states(1, 0, B)
    s = sm.BatchSolver(N, 2 * N, B, dtype=dt)
    s.setup(ops["P"], np.zeros(N), ops["A"], np.full(2 * N, -np.finfo(float).max), ops["W0"])
    s.mpc_set_operators(ops["Fx"], ops["Fu"], ops["Fr"], ops["Sbar"], ops["Ku"], ops["W0"])
    s.mpc_set_plant(plant["Ad"], plant["Bd"])
    Xd = torch.from_numpy(X).cuda()
    Ud = torch.from_numpy(U).cuda()
    st = torch.cuda.Stream()
    for chunk in range(6):
        with torch.cuda.stream(st):
            s.mpc_run_device(Xd.data_ptr(), Ud.data_ptr(), 0.0, 50, 1, 0, chunk * 50, 1e-2, st.cuda_stream)
        st.synchronize()
        stt, it, rho = s.info()
        vals, cnt = np.unique(stt, return_counts=True)
        Xh = Xd.cpu().numpy()
        print(dt, (chunk + 1) * 50, dict(zip(vals.tolist(), cnt.tolist())), "iters mean %.1f" % it.mean(),
              "max|X| %.3g" % np.abs(Xh).max(), "argmax", int(np.abs(Xh).max(1).argmax()),
              "max|U| %.3g" % np.abs(Ud.cpu().numpy()).max(), flush=True)
    s.close()
