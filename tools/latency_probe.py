"""Dev tool (GPU): per-iteration latency of a lone wave on each device path.  A batch of 16 shared-plant
QPs (one tile wave) or 2 per-plant QPs (one plant_step wave) runs a fixed number of iterations (eps = 0:
no convergence; max_iter = K) and the solve time / K is printed."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import solvempc_amd as sm  # noqa: E402
from solvempc_amd import workload  # noqa: E402

N, K = 20, int(os.environ.get("K", "400"))
dev = torch.device("cuda:0")
plant = workload.reference_plant()
ops = sm.mpc.condense({"Ad": plant["Ad"][None], "Bd": plant["Bd"][None], "Cd": plant["Cd"][None],
                       "K": plant["K"][None], "Q": [plant["Q"]], "R": [plant["R"]], "RD": [plant["RD"]]}, N, device=0)
ops = {k: v[0] for k, v in ops.items()}
stream = torch.cuda.current_stream(dev)


def timed(fn, reps=10):
    ts = []
    for i in range(reps + 2):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        fn()
        e1.record(stream)
        torch.cuda.synchronize()
        if i >= 2:
            ts.append(e0.elapsed_time(e1))
    return float(np.median(ts))


for dtype in ("f32", "f64"):
    st = sm.default_settings(eps_abs=1e-15, eps_rel=1e-15, max_iter=K, adaptive_rho=0)
    for kern, B in (("tile", 16), ("tile", 8192), ("wave", 16)):
        os.environ["MPCQ_KERNEL"] = kern
        os.environ["MPCQ_PHASES"] = "0"
        X, U = workload.mpc_states(1, 0, B)
        s = sm.BatchSolver(N, 2 * N, B, 1, dtype, 0, settings=st)
        s.setup(ops["P"], np.zeros(N), ops["A"], np.full(2 * N, -np.finfo(np.float64).max), ops["W0"].copy())
        s.mpc_set_operators(ops["Fx"], ops["Fu"], ops["Fr"], ops["Sbar"], ops["Ku"], ops["W0"])
        Xd, Ud = torch.from_numpy(X).to(dev), torch.from_numpy(U).to(dev)

        def run():
            s.reset_state()
            s.mpc_step_device(Xd.data_ptr(), Ud.data_ptr(), 0.0, stream.cuda_stream)
        ms = timed(run)
        _, it, _ = s.info()
        print(f"{dtype} {kern:5s} B={B:5d} path={s.path()} iters {it.max()}  {ms * 1e3 / K:.3f} us/iteration", flush=True)
        s.close()
    os.environ.pop("MPCQ_KERNEL", None)
    os.environ.pop("MPCQ_PHASES", None)
    # per-plant one-pass kernel: 2 plants = one wave
    B = 2
    Ad, Bd = workload.randomized_plants(plant, 2, 0, B)
    X, U = workload.mpc_states(2, 0, B)
    t = lambda v: torch.as_tensor(np.ascontiguousarray(v, dtype=np.float64), device=dev)  # noqa: E731
    pl = [t(Ad), t(Bd), t(np.tile(plant["Cd"], (B, 1))), t(np.tile(plant["K"], (B, 1))), t(np.full(B, plant["Q"])),
          t(np.full(B, plant["R"])), t(np.full(B, plant["RD"]))]
    Xd, U0 = t(X), t(U)
    s = sm.BatchSolver(N, 2 * N, B, n_plants=B, dtype=dtype, settings=st)
    ms_k = timed(lambda: s.mpc_plants_step_device(4, 10, *[x.data_ptr() for x in pl], Xd.data_ptr(), U0.clone().data_ptr()))
    s.close()
    s = sm.BatchSolver(N, 2 * N, B, n_plants=B, dtype=dtype, settings=sm.default_settings(eps_abs=1e-15, eps_rel=1e-15, max_iter=1, adaptive_rho=0))
    ms_1 = timed(lambda: s.mpc_plants_step_device(4, 10, *[x.data_ptr() for x in pl], Xd.data_ptr(), U0.clone().data_ptr()))
    s.close()
    print(f"{dtype} plant B=2 {(ms_k - ms_1) * 1e3 / (K - 1):.3f} us/iteration (setup + 1 iteration {ms_1 * 1e3:.1f} us)", flush=True)
