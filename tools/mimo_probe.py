"""Config-4 solve-kernel probe (dev tool): solve-stage time for settings variants (max_iter, adaptive
rho off) on a slice of the quad-rotor batch, and MPCQ_MIMO_STAMPS per-QP stage cycles.
usage: python tools/mimo_probe.py [batch]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import solvempc_amd as sm  # noqa: E402
from solvempc_amd import workload  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
N, nu = 30, 4
Ad, Bd = workload.quadrotor_plants(3, 0, B)
sh = workload.quadrotor_shared()
X, U = workload.quadrotor_states(3, 0, B)
dev = torch.device("cuda", 0)
td = lambda v: torch.as_tensor(np.ascontiguousarray(v, dtype=np.float64)).to(dev)  # noqa: E731
pd = [td(Ad), td(Bd)] + [td(np.broadcast_to(np.asarray(sh[k], dtype=np.float64), (B,) + np.asarray(sh[k]).shape))
                         for k in ("Cd", "Q", "R", "RD", "K", "K0", "w0")]
Xd, U0 = td(X), td(U)
stream = torch.cuda.current_stream(dev)


def run(label, stamps=None, **over):
    s = sm.BatchSolver(N * nu, 2 * N * nu, B, B, "f64", 0, settings=sm.default_settings(**over))
    Ud = U0.clone()
    times = []
    for rep in range(3):
        s.mimo_setup_plants_device(12, nu, 12, N, *[t.data_ptr() for t in pd], stream=stream.cuda_stream)
        Ud.copy_(U0)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if stamps and rep == 2:
            os.environ["MPCQ_MIMO_STAMPS"] = stamps
        e0.record(stream)
        s.mimo_step_device(Xd.data_ptr(), Ud.data_ptr(), 0, stream.cuda_stream)
        e1.record(stream)
        torch.cuda.synchronize()
        os.environ.pop("MPCQ_MIMO_STAMPS", None)
        times.append(e0.elapsed_time(e1))
    st, it, rho = s.info()
    print(f"{label:34s} solve {min(times):9.2f} ms  iters mean {it.mean():6.1f} max {it.max():4d}  "
          f"us/QP/CU {min(times) * 1e3 / (B / 256):8.2f}", flush=True)
    if stamps:
        r = np.fromfile(stamps, dtype=np.int64).reshape(B, 8)
        fe, inv, tot = r[:, 1] - r[:, 0], r[:, 2] - r[:, 1], r[:, 3] - r[:, 0]
        loop = r[:, 3] - r[:, 2]
        print(f"   cycles (median): front {np.median(fe):.0f} first-invert {np.median(inv):.0f} "
              f"after-last-invert {np.median(loop):.0f} total {np.median(tot):.0f}; iters {np.median(r[:, 4]):.0f}",
              flush=True)
    s.close()


if len(sys.argv) > 2 and sys.argv[2] == "setup":
    os.environ["MPCQ_MIMO_SETUP_STAMPS"] = "gpurun_out/setup_stamps.bin"
    run("setup stamps", max_iter=1, adaptive_rho=0)
    sys.exit(0)
run("max_iter 1, no adapt", max_iter=1, adaptive_rho=0, stamps="gpurun_out/ms1.bin")
if len(sys.argv) > 2 and sys.argv[2] == "gj":
    sys.exit(0)
run("max_iter 25, no adapt", max_iter=25, adaptive_rho=0, stamps="gpurun_out/ms25.bin")
run("max_iter 100, no adapt", max_iter=100, adaptive_rho=0, check_termination=0)
run("default", stamps="gpurun_out/msd.bin")
