"""bench.py — BASELINE.json metric: QP solves/sec for the condensed MPC QP (n_x=4, n_u=1, N=20),
config 2 at N=1: a batch of 65,536 copies of the reference controller (identical plant, per-QP
state X ~ N(0, diag(.1,.1,.05,.5)), U ~ U(-1,1)), solved on MI355X.

One step = one ModelPredictiveControlAPI::controllerStep (src/ModelPredictiveControlAPI.cpp:81-108)
for every QP of the batch, from the post-setup solver state (the reference's first control step):
q and u built on the device from (X, U), OSQP-v0.6 ADMM solve, U += x[0].  Inputs are resident in
HBM before timing.  Multi-GPU: one process per GPU, each rank solves its own 65,536 QPs (weak
scaling, shards of one counter-based global stream) and the applied moves are gathered to rank 0
over RCCL (the path's only exchange).  Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

# MI355X dense matrix-core peaks (MI355X_MICROARCH.md: f32-input MFMA 157.3 TF = the f32 vector
# peak; f64 78.6 TF).  The tile kernel's three ADMM products run on the matrix pipe.
PEAK_TFLOPS = {"f64": 78.6, "f32": 157.3}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--batch", type=int, default=65536, help="QPs per GPU")
    p.add_argument("--horizon", type=int, default=20)
    p.add_argument("--dtype", choices=("f64", "f32"), default="f32", help="ADMM iterate type (BASELINE cfg 2: fp32)")
    p.add_argument("--seed", type=int, default=1)
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline budget (0 = skip)")
    p.add_argument("--cpu-threads", type=int, default=0)
    p.add_argument("--workload", choices=("cfg2", "stream", "perplant", "quadrotor"), default="cfg2",
                   help="cfg2: BASELINE config 2 (the headline); stream: config 5 (4,096 plants x --ctrl-steps "
                        "warm-started control steps with a simulated plant, hipGraph-replayed); perplant: config 3 "
                        "(randomised plants, per-GPU shard of 1M: condense + setup + one controllerStep each); "
                        "quadrotor: config 4 (262,144 quad-rotor hover linearisations, n_x 12, n_u 4, N 30: MIMO "
                        "condense + setup + one controllerStep each, fp64)")
    p.add_argument("--ctrl-steps", type=int, default=1000, help="control steps per bench step (stream)")
    p.add_argument("--noise", type=float, default=1e-2, help="plant noise std (stream; SURVEY §8d: var 1e-4)")
    a = p.parse_args()
    if a.workload == "stream" and a.batch == 65536:
        a.batch = 4096
    if a.workload == "perplant" and a.batch == 65536:
        a.batch = 131072  # 1,048,576 / 8 GPUs
        if a.seed == 1:
            a.seed = 2  # SURVEY §8d config 3 seed
    if a.workload == "quadrotor":
        if a.batch == 65536:
            a.batch = 262144  # BASELINE config 4
        if a.horizon == 20:
            a.horizon = 30
        if a.seed == 1:
            a.seed = 3  # SURVEY §8d config 4 seed
        a.dtype = "f64"
    return a


def cpu_baseline(ops, N, X, U, budget_s, threads):
    """The oracle (fp64 C restatement of OSQP-0.6, OpenMP) on a bounded sample of the same workload."""
    import oracle

    l = np.full(2 * N, -np.finfo(np.float64).max)
    q0, u0 = np.zeros(N), oracle.upper_bound(ops, np.zeros(4), 0.0)
    q, u = oracle.gradient(ops, X, U), oracle.upper_bound(ops, X, U)
    nthr = threads or min(16, os.cpu_count() or 1)
    n = 256
    while True:
        t0 = time.perf_counter()
        oracle.batch_solve(ops["P"], ops["A"], q0, l, u0, q[:n], u[:n], nthreads=nthr)
        dt = time.perf_counter() - t0
        if dt > budget_s / 4 or n >= len(X):
            break
        n = min(len(X), int(n * max(2.0, budget_s / 4 / max(dt, 1e-3))))
    return {"value": n / dt, "unit": "QP/s", "cores": nthr, "kind": "port",
            "sample": f"{n} QPs of the same batch (first {n} states), oracle/osqp_dense.c fp64, "
                      f"OpenMP {nthr} threads, {dt:.2f} s"}


def cpu_baseline_plants(plant, Ad, Bd, N, X, U, budget_s, threads):
    """The oracle's per-plant path (condense + setup + one controllerStep, fp64 C, OpenMP) on a
    bounded sample of the config-3 plants."""
    import oracle

    nthr = threads or min(16, os.cpu_count() or 1)
    n = 256
    while True:
        t0 = time.perf_counter()
        oracle.plants_step(plant, Ad[:n], Bd[:n], X[:n], U[:n], N, nthreads=nthr)
        dt = time.perf_counter() - t0
        if dt > budget_s / 4 or n >= len(X):
            break
        n = min(len(X), int(n * max(2.0, budget_s / 4 / max(dt, 1e-3))))
    return {"value": n / dt, "unit": "QP/s", "cores": nthr, "kind": "port",
            "sample": f"{n} plants of the same batch (first {n}): oracle/mpc_batch.c condense + osqp_dense.c "
                      f"setup + solve, fp64, OpenMP {nthr} threads, {dt:.2f} s"}


def cpu_baseline_quadrotor(shared, Ad, Bd, X, U, N, budget_s, threads):
    """The oracle's MIMO per-plant path (condense + OSQP-0.6 setup + one controllerStep, fp64 C,
    OpenMP) on a bounded sample of the config-4 plants."""
    import oracle

    nthr = threads or min(16, os.cpu_count() or 1)
    n = 64
    while True:
        t0 = time.perf_counter()
        oracle.mimo_plants_step(shared, Ad[:n], Bd[:n], X[:n], U[:n], N, nthreads=nthr)
        dt = time.perf_counter() - t0
        if dt > budget_s / 4 or n >= len(X):
            break
        n = min(len(X), int(n * max(2.0, budget_s / 4 / max(dt, 1e-3))))
    return {"value": n / dt, "unit": "QP/s", "cores": nthr, "kind": "port",
            "sample": f"{n} plants of the same batch (first {n}): oracle/mpc_mimo.c condense + osqp_dense.c "
                      f"setup + solve, fp64, OpenMP {nthr} threads, {dt:.2f} s"}


def main_quadrotor(a, rank, world, local, dist, dev):
    """BASELINE config 4: every QP its own quad-rotor plant (hover linearisation with +-10% mass and
    inertia, ZOH dt 0.02); one step = device condensing + setup of every plant + one controllerStep
    each (mpcq_mimo_setup_plants_device + mpcq_mimo_step_device), fp64."""
    import torch

    import solvempc_amd as sm
    from solvempc_amd import dist as mdist
    from solvempc_amd import workload

    N, B = a.horizon, a.batch
    nu = 4
    start, count = mdist.weak_block(B, rank)
    Ad, Bd = workload.quadrotor_plants(a.seed, start, count)
    sh = workload.quadrotor_shared()
    X, U = workload.quadrotor_states(a.seed, start, count)
    nx, ny = Ad.shape[1], np.asarray(sh["Cd"]).shape[0]
    tdev = lambda v: torch.as_tensor(np.ascontiguousarray(v, dtype=np.float64)).to(dev)  # noqa: E731
    plant_d = [tdev(Ad), tdev(Bd)] + [
        torch.as_tensor(np.asarray(sh[k], dtype=np.float64)).to(dev).expand((B,) + np.asarray(sh[k]).shape).contiguous()
        for k in ("Cd", "Q", "R", "RD", "K", "K0", "w0")]
    solver = sm.BatchSolver(N * nu, 2 * N * nu, B, B, "f64", local)
    X_d, U0_d = tdev(X), tdev(U)
    U_d = U0_d.clone()
    stream = torch.cuda.current_stream(dev)
    sptr = stream.cuda_stream
    gathered = [torch.empty_like(U_d) for _ in range(world)] if rank == 0 else None

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
    ev_mid = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps)]

    def step(i=None):
        U_d.copy_(U0_d)  # the reference's first control step of each plant (setup resets the solver)
        if i is not None:
            ev[i][0].record(stream)
        solver.mimo_setup_plants_device(nx, nu, ny, N, *[t.data_ptr() for t in plant_d], stream=sptr)
        if i is not None:
            ev_mid[i].record(stream)
        solver.mimo_step_device(X_d.data_ptr(), U_d.data_ptr(), 0, sptr)
        if i is not None:
            ev[i][1].record(stream)
        mdist.gather_moves(dist, U_d, world, rank, gathered)

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([wall], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall = float(t.item())
    kern_ms = float(np.mean([s.elapsed_time(e) for s, e in ev]))
    setup_ms = float(np.mean([s.elapsed_time(m_) for (s, _), m_ in zip(ev, ev_mid)]))
    solve_ms = float(np.mean([m_.elapsed_time(e) for (_, e), m_ in zip(ev, ev_mid)]))
    status, iters, rho = solver.info()
    n = N * nu
    # factorisations: the initial inverse plus (at least) one per QP whose rho moved
    fact = 1 + (rho != solver.settings.rho)
    setup_flops = B * workload.flops_mimo_setup(N, nx, nu, ny, solver.settings.scaling)
    solve_flops = float(workload.flops_mimo_solve(n, nu, iters, fact).sum())
    dense = float(workload.flops_mimo_dense(N, nx, nu, ny, iters).sum())
    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return
    tf = lambda f, ms: f / (ms * 1e-3) / 1e12  # noqa: E731
    peak = PEAK_TFLOPS["f64"]
    rec = {
        "metric": "QP solves/sec (quad-rotor n_x=12, n_u=4, N=30 batch)",
        "value": B * world * a.steps / wall,
        "unit": "QP/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": wall / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (hover linearisations, mass/inertia +-10% counter-based per plant; X ~ N(0, diag), U ~ U(-w0/2, w0/2))",
        "config": {"workload": f"cfg4: {B} quad-rotor plants per GPU (n_x {nx}, n_u {nu}, n_y {ny}), N={N} "
                               f"(n={n}, m={2 * n}): on-device MIMO condensing + setup + one controllerStep each",
                   "batch_per_gpu": B, "horizon": N, "parallelism": f"dp{world}"},
        # dominant stage: the per-QP solve (Gauss-Jordan KKT inverse + ADMM iterations, fp64 VALU)
        "roofline": {"bound": "valu", "achieved": tf(solve_flops, solve_ms), "peak": peak, "unit": "TFLOP/s",
                     "frac": tf(solve_flops, solve_ms) / peak, "traffic": None,
                     "kernel": "mimo_solve_kernel (fp64 vector peak)", "kernel_ms": solve_ms,
                     "flops_per_step": solve_flops,
                     "flops_note": "algorithmic for the structured solve: 2n^3 per KKT inverse (1 + one per QP whose "
                                   "rho adapted), iters x (2n^2 + structured A products + 30n) "
                                   "(workload.flops_mimo_solve)"},
        "stages": {"setup_ms": setup_ms, "solve_ms": solve_ms, "step_ms": kern_ms,
                   "setup_roofline": {"bound": "valu", "achieved": tf(setup_flops, setup_ms), "peak": peak,
                                      "unit": "TFLOP/s", "frac": tf(setup_flops, setup_ms) / peak,
                                      "kernel": "mimo_setup_kernel", "flops_per_step": setup_flops,
                                      "note": "timed span includes the host read-back of the setup status word"}},
        "dense_equivalent": {"flops_per_step": dense, "achieved": tf(dense, kern_ms), "frac": tf(dense, kern_ms) / peak,
                             "note": "SURVEY §8d count: dense condensing + Ruiz + one KKT LDL + iters x F_iter(n, m)"},
        "iters": {"mean": float(iters.mean()), "max": int(iters.max()),
                  "solved_frac": float(np.mean(status == sm.SOLVED)), "rho_adapted_frac": float(np.mean(fact > 1))},
    }
    if a.cpu_seconds > 0:
        rec["cpu_baseline"] = cpu_baseline_quadrotor(sh, Ad, Bd, X, U, N, a.cpu_seconds, a.cpu_threads)
    print(json.dumps(rec))
    if dist:
        dist.destroy_process_group()


def traffic_per_solve(dtype, batch, N):
    """HBM bytes of one solve from the committed PMC pass (tools/pmc.sh -> profiles/), or None."""
    f = ROOT / "profiles" / f"pmc_traffic_{dtype}.json"
    try:
        d = json.loads(f.read_text())
    except (OSError, ValueError):
        return None
    if d.get("batch") != batch or d.get("horizon") != N:
        return None
    return d.get("bytes_per_solve")


def main():
    a = parse()
    from solvempc_amd import dist as mdist

    rank, world, local = mdist.world_from_env(a.gpus)
    import torch

    dist = None
    if world > 1:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", rank=rank, world_size=world)
    else:
        torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if a.workload == "quadrotor":
        return main_quadrotor(a, rank, world, local, dist, dev)

    import solvempc_amd as sm
    from solvempc_amd import workload

    N, B = a.horizon, a.batch
    plant = workload.reference_plant()
    ops = sm.mpc.condense({"Ad": plant["Ad"][None], "Bd": plant["Bd"][None], "Cd": plant["Cd"][None],
                           "K": plant["K"][None], "Q": [plant["Q"]], "R": [plant["R"]], "RD": [plant["RD"]]},
                          N, device=local)
    ops = {k: v[0] for k, v in ops.items()}
    start, count = mdist.weak_block(B, rank)  # weak scaling: every rank owns B QPs of the global stream
    X, U = workload.mpc_states(a.seed, start, count)
    l = np.full(2 * N, -np.finfo(np.float64).max)
    u0 = ops["W0"].copy()  # W0 + Sbar 0 + Ku 0 (:43)

    perplant = a.workload == "perplant"
    if perplant:  # config 3: every QP its own plant, condensed and set up on the device each step
        Ad, Bd = workload.randomized_plants(plant, a.seed, start, count)
        solver = sm.BatchSolver(N, 2 * N, B, B, a.dtype, local)
        tdev = lambda v: torch.as_tensor(np.ascontiguousarray(v, dtype=np.float64)).to(dev)  # noqa: E731
        plant_d = [tdev(Ad), tdev(Bd), tdev(np.tile(plant["Cd"], (B, 1))), tdev(np.tile(plant["K"], (B, 1))),
                   tdev(np.full(B, plant["Q"])), tdev(np.full(B, plant["R"])), tdev(np.full(B, plant["RD"]))]
    else:
        solver = sm.BatchSolver(N, 2 * N, B, 1, a.dtype, local)
        solver.setup(ops["P"], np.zeros(N), ops["A"], l, u0)
        solver.mpc_set_operators(ops["Fx"], ops["Fu"], ops["Fr"], ops["Sbar"], ops["Ku"], ops["W0"])
    X_d = torch.from_numpy(X).to(dev)
    U0_d = torch.from_numpy(U).to(dev)
    U_d = U0_d.clone()
    stream = torch.cuda.current_stream(dev)
    sptr = stream.cuda_stream
    gathered = [torch.empty_like(U_d) for _ in range(world)] if rank == 0 else None

    stream_mode = a.workload == "stream"
    if stream_mode:
        solver.mpc_set_plant(plant["Ad"], plant["Bd"])
        side = torch.cuda.Stream(dev)  # graph capture needs a non-default stream
        stream, sptr = side, side.cuda_stream
        X0_d = X_d.clone()
    ctrl_base = [0]

    def launch(i=None):
        if stream_mode:  # config 5: ctrl_steps warm-started control steps + plant updates (hipGraph)
            solver.mpc_run_device(X_d.data_ptr(), U_d.data_ptr(), plant["xref"], a.ctrl_steps, a.seed, start,
                                  ctrl_base[0], a.noise, sptr)
            ctrl_base[0] += a.ctrl_steps
        else:
            if perplant:  # condensing + Ruiz + eigen-basis setup of every plant, on the device
                solver.mpc_setup_plants_device(4, 10, *[t.data_ptr() for t in plant_d], sptr)
                if i is not None:
                    ev_mid[i].record(stream)  # setup | solve boundary (same stream)
            solver.mpc_step_device(X_d.data_ptr(), U_d.data_ptr(), plant["xref"], sptr)

    def reset():
        U_d.copy_(U0_d)          # every step: the reference's first control step of each plant
        if not perplant:         # (perplant: the setup inside the step resets the state)
            solver.reset_state()  # post-setup solver state (x = z = y = 0, rho = settings.rho)
        if stream_mode:
            X_d.copy_(X0_d)
            ctrl_base[0] = 0

    cur = torch.cuda.current_stream(dev)

    def step(i=None):
        reset()
        if stream_mode:
            stream.wait_stream(cur)  # the resets above ran on the current stream
        if i is not None:
            ev[i][0].record(stream)
        launch(i)
        if i is not None:
            ev[i][1].record(stream)
        if stream_mode:
            cur.wait_stream(stream)
        mdist.gather_moves(dist, U_d, world, rank, gathered)

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
    ev_mid = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps)]
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([wall], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall = float(t.item())
    kern_ms = float(np.mean([s.elapsed_time(e) for s, e in ev]))
    if perplant:
        setup_ms = float(np.mean([s.elapsed_time(m_) for (s, _), m_ in zip(ev, ev_mid)]))
        solve_ms = float(np.mean([m_.elapsed_time(e) for (_, e), m_ in zip(ev, ev_mid)]))

    status, iters, _ = solver.info()
    qps_per_step = B * (a.ctrl_steps if stream_mode else 1)
    # stream: iterations of the last control step stand for every step (estimate, see "flops_note")
    kind, paired = solver.path()
    reps = a.ctrl_steps if stream_mode else 1
    flops = float(workload.flops_per_qp(N, 2 * N, 4, iters, paired=paired).sum()) * reps
    flops_dense = float(workload.flops_per_qp(N, 2 * N, 4, iters).sum()) * reps
    achieved = flops / (kern_ms * 1e-3) / 1e12
    if perplant:
        setup_flops = B * workload.flops_plant_setup(N, 2 * N)
    solved = float(np.mean(status == sm.SOLVED))

    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return
    total_qps = qps_per_step * world * a.steps / wall
    rec = {
        "metric": "QP solves/sec (n_x=4, n_u=1, N=20 batch)",
        "value": total_qps,
        "unit": "QP/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": wall / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": a.dtype,
        "data": "synthetic (counter-based X ~ N(0, diag(.1,.1,.05,.5)), U ~ U(-1,1); reference plant config)",
        "config": ({"workload": f"cfg2: {B} identical LTI plants per GPU, N={N} (n={N}, m={2 * N}), "
                                f"one controllerStep each", "batch_per_gpu": B, "horizon": N,
                    "parallelism": f"dp{world}"} if a.workload == "cfg2" else
                   {"workload": f"cfg3: {B} randomised plants per GPU (Ad, Bd +-2% ~ N(0,1), rho(Ad) < 1), N={N}: "
                                f"on-device condensing + setup + one controllerStep each",
                    "batch_per_gpu": B, "horizon": N, "parallelism": f"dp{world}"} if perplant else
                   {"workload": f"cfg5: {B} plants per GPU x {a.ctrl_steps} warm-started control steps, "
                                f"simulated plant (noise std {a.noise}), hipGraph-replayed, N={N}",
                    "batch_per_gpu": B, "horizon": N, "ctrl_steps": a.ctrl_steps, "parallelism": f"dp{world}"}),
        "roofline": {"bound": "mfma", "achieved": achieved, "peak": PEAK_TFLOPS[a.dtype], "unit": "TFLOP/s",
                     "frac": achieved / PEAK_TFLOPS[a.dtype], "traffic": traffic_per_solve(a.dtype, B, N),
                     "kernel": f"admm_{kind}_kernel{' (paired loop)' if paired else ''} (all phase launches of one solve)",
                     "kernel_ms": kern_ms, "flops_per_step": flops,
                     "dense_equivalent": {"flops_per_step": flops_dense,
                                          "achieved": flops_dense / (kern_ms * 1e-3) / 1e12,
                                          "frac": flops_dense / (kern_ms * 1e-3) / 1e12 / PEAK_TFLOPS[a.dtype]},
                     "flops_note": "algorithmic: sum over QPs of iters*F_iter + checks*F_check + front end "
                                   "(SURVEY §8d, DESIGN §4.1), actual per-QP iteration counts"
                                   + ("; F_iter counts the m/2-row products the paired loop performs "
                                      "(dense_equivalent: the dense 4nm count)" if paired else "")
                                   + ("; stream: last control step's counts x ctrl_steps (estimate)" if stream_mode else "")},
        "iters": {"mean": float(iters.mean()), "max": int(iters.max()), "solved_frac": solved},
    }
    if perplant:
        # The step is two stages of different character: per-plant condensing + setup (fp64 VALU/LDS,
        # one wave per plant; the dominant stage) and the one-QP-per-wave ADMM solve (VALU, T = dtype).
        # Each is priced against its own vector peak; the timed span of the setup stage includes the
        # host read-back of the setup status word (mpcq_mpc_setup_plants_device synchronises once).
        rec["roofline"] = {"bound": "valu", "achieved": setup_flops / (setup_ms * 1e-3) / 1e12,
                           "peak": PEAK_TFLOPS["f64"], "unit": "TFLOP/s",
                           "frac": setup_flops / (setup_ms * 1e-3) / 1e12 / PEAK_TFLOPS["f64"], "traffic": None,
                           "kernel": "condense_wave_kernel + setup_wave_kernel (fp64 vector peak)",
                           "kernel_ms": setup_ms, "flops_per_step": setup_flops,
                           "flops_note": "algorithmic per plant (SURVEY §8d): F_condense + Ruiz + one LDL of the "
                                         "KKT system; the eigen-basis setup's extra work is not credited"}
        rec["stages"] = {"setup_ms": setup_ms, "solve_ms": solve_ms, "step_ms": kern_ms,
                         "solve_roofline": {"bound": "valu", "achieved": flops / (solve_ms * 1e-3) / 1e12,
                                            "peak": PEAK_TFLOPS[a.dtype], "unit": "TFLOP/s",
                                            "frac": flops / (solve_ms * 1e-3) / 1e12 / PEAK_TFLOPS[a.dtype],
                                            "kernel": "admm_wave_kernel", "flops_per_step": flops}}
    if a.cpu_seconds > 0 and perplant:
        rec["cpu_baseline"] = cpu_baseline_plants(plant, Ad, Bd, N, X, U, a.cpu_seconds, a.cpu_threads)
    elif a.cpu_seconds > 0 and not stream_mode:
        rec["cpu_baseline"] = cpu_baseline(ops, N, X, U, a.cpu_seconds, a.cpu_threads)
    print(json.dumps(rec))
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
