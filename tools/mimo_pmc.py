"""One config-4 setup + solve launch for PMC passes (dev tool).
usage: python tools/mimo_pmc.py {gj|iter|full} [batch]
gj: max_iter 1, adaptive rho off (the Gauss-Jordan inverse dominates); iter: max_iter 100, no
checks, adaptive rho off (the iterations dominate); full: default settings."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import solvempc_amd as sm  # noqa: E402
from solvempc_amd import workload  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "full"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
N, nu = 30, 4
over = {"gj": dict(max_iter=1, adaptive_rho=0), "iter": dict(max_iter=100, adaptive_rho=0, check_termination=0),
        "full": {}}[mode]
Ad, Bd = workload.quadrotor_plants(3, 0, B)
sh = workload.quadrotor_shared()
X, U = workload.quadrotor_states(3, 0, B)
dev = torch.device("cuda", 0)
td = lambda v: torch.as_tensor(np.ascontiguousarray(v, dtype=np.float64)).to(dev)  # noqa: E731
pd = [td(Ad), td(Bd)] + [td(np.broadcast_to(np.asarray(sh[k], dtype=np.float64), (B,) + np.asarray(sh[k]).shape))
                         for k in ("Cd", "Q", "R", "RD", "K", "K0", "w0")]
s = sm.BatchSolver(N * nu, 2 * N * nu, B, B, "f64", 0, settings=sm.default_settings(**over))
stream = torch.cuda.current_stream(dev).cuda_stream
s.mimo_setup_plants_device(12, nu, 12, N, *[t.data_ptr() for t in pd], stream=stream)
Xd, Ud = td(X), td(U)
s.mimo_step_device(Xd.data_ptr(), Ud.data_ptr(), 0, stream)
torch.cuda.synchronize()
st, it, _ = s.info()
print(mode, B, "iters mean", float(it.mean()))
