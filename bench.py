"""bench.py — BASELINE.json metric: QP solves/sec for the condensed MPC QP (n_x=4, n_u=1, N=20),
config 2 at N=1: a batch of 65,536 copies of the reference controller (identical plant, per-QP
state X ~ N(0, diag(.1,.1,.05,.5)), U ~ U(-1,1)), solved on MI355X.

One step = one ModelPredictiveControlAPI::controllerStep (src/ModelPredictiveControlAPI.cpp:81-108)
for every QP of the batch, from the post-setup solver state (the reference's first control step):
q and u built on the device from (X, U), OSQP-v0.6 ADMM solve, U += x[0].  Inputs are resident in
HBM before timing.  Multi-GPU: one process per GPU, each rank solves its own 65,536 QPs (weak
scaling, shards of one counter-based global stream) and the applied moves are gathered to rank 0
over RCCL (the path's only exchange).  Prints ONE JSON line on rank 0.

`python bench.py --gpus N` starts its own N ranks (one process per GPU, spawned before anything
touches a GPU) unless a launcher (torch.distributed.run) already set RANK / WORLD_SIZE.
`--backend gloo --dry-run` runs the launcher and the gather on the CPU without a device (tests).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

# MI355X dense matrix-core peaks (MI355X_MICROARCH.md: f32-input MFMA 157.3 TF = the f32 vector
# peak; f64 78.6 TF).  The tile kernel's three ADMM products run on the matrix pipe.
PEAK_TFLOPS = {"f64": 78.6, "f32": 157.3}
# The mixed tile path (MPCQ_F64_MIXED) performs each FLOP in one of the two types: its peak is the rate
# at which the matrix cores would perform that split, 1 / (share64 / 78.6 + share32 / 157.3).
DTYPE_NAME = {"f64": "f64", "f32": "f32", "mixed": "f64+f32 (mixed: fp64 state, checks and solution; fp32 plain iterations)"}


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--batch", type=int, default=65536, help="QPs per GPU")
    p.add_argument("--horizon", type=int, default=20)
    p.add_argument("--dtype", choices=("f64", "f32", "mixed"), default=None,
                   help="ADMM arithmetic (default: the fastest path inside north_star's 1e-5 on the applied move: "
                        "mixed for cfg2, f64 for perplant (faster than its fp32 kernel, which misses it) and for the "
                        "stream (whose mixed / f32 closed loops drift up to ~3e-5 from the oracle's over 1,000 "
                        "steps); quadrotor is f64)")
    p.add_argument("--variants", type=int, default=1,
                   help="cfg2: also time the f32 and f64 paths on the same batch (the line's `variants` block)")
    p.add_argument("--seed", type=int, default=1)
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline budget (0 = skip)")
    p.add_argument("--cpu-threads", type=int, default=0, help="threads of the multi-threaded CPU leg (0: all usable)")
    p.add_argument("--workload", choices=("cfg2", "stream", "perplant", "quadrotor"), default="cfg2",
                   help="cfg2: BASELINE config 2 (the headline); stream: config 5 (4,096 plants x --ctrl-steps "
                        "warm-started control steps with a simulated plant, hipGraph-replayed); perplant: config 3 "
                        "(randomised plants, per-GPU shard of 1M: condense + setup + one controllerStep each); "
                        "quadrotor: config 4 (262,144 quad-rotor hover linearisations, n_x 12, n_u 4, N 30: MIMO "
                        "condense + setup + one controllerStep each, fp64)")
    p.add_argument("--scaling", choices=("weak", "strong"), default="weak",
                   help="weak: --batch QPs per GPU; strong: one global batch (--global-batch) split over the GPUs "
                        "(dist.strong_block); BASELINE config 3 is `--workload perplant --scaling strong`")
    p.add_argument("--global-batch", type=int, default=0,
                   help="strong scaling: QPs of the whole job (default: 1,048,576 for perplant, else --batch)")
    p.add_argument("--cfg3-strong", type=int, default=1,
                   help="cfg2 line: also run BASELINE config 3 as written -- ONE batch of --cfg3-global-batch "
                        "randomised plants split over the N ranks, RCCL gather of U to rank 0 -- and report it as "
                        "the line's `cfg3_strong` block (0 = skip)")
    p.add_argument("--cfg3-global-batch", type=int, default=1 << 20, help="plants of the cfg3_strong job")
    p.add_argument("--ctrl-steps", type=int, default=1000, help="control steps per bench step (stream)")
    p.add_argument("--noise", type=float, default=1e-2, help="plant noise std (stream; SURVEY §8d: var 1e-4)")
    p.add_argument("--backend", choices=("nccl", "gloo"), default="nccl",
                   help="torch.distributed backend of the gather (nccl = RCCL on ROCm)")
    p.add_argument("--dry-run", action="store_true",
                   help="no device: launcher, rendezvous and the gather only (CPU tests of the N > 1 plumbing)")
    a = p.parse_args(argv)
    if a.dtype is None:  # the fastest path inside north_star's 1e-5 on the applied move
        a.dtype = {"cfg2": "mixed", "perplant": "f64", "stream": "f64"}.get(a.workload, "f32")
    if a.workload == "stream" and a.batch == 65536:
        a.batch = 4096
    if a.workload == "perplant":
        if a.batch == 65536:
            a.batch = 131072  # 1,048,576 / 8 GPUs
        if a.seed == 1:
            a.seed = 2  # SURVEY §8d config 3 seed (weak and strong alike)
    if a.scaling == "strong" and not a.global_batch:
        a.global_batch = 1 << 20 if a.workload == "perplant" else a.batch  # BASELINE config 3: 1,048,576 plants
    if a.workload == "stream" and a.seed == 1:
        a.seed = 4  # SURVEY §8d config 5 seed
    if a.workload == "quadrotor":
        if a.batch == 65536:
            a.batch = 262144  # BASELINE config 4
        if a.horizon == 20:
            a.horizon = 30
        if a.seed == 1:
            a.seed = 3  # SURVEY §8d config 4 seed
        a.dtype = "f64"
    return a


# ----------------------------------------------------------------------------- launcher
def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(a, argv) -> int:
    """One process per GPU, started before anything in this process touches a GPU.  Each child gets
    torch.distributed.run's environment (RANK, LOCAL_RANK, WORLD_SIZE, MASTER_ADDR, MASTER_PORT);
    rank 0's JSON line is relayed.  Returns the worst child exit code."""
    import threading

    port = _free_port()
    procs = []
    for r in range(a.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.gpus), LOCAL_WORLD_SIZE=str(a.gpus),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(Path(__file__).resolve())] + argv, env=env,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL, text=True))
    out = []
    reader = threading.Thread(target=lambda: out.append(procs[0].stdout.read()), daemon=True)
    reader.start()
    # poll every rank: the first one to fail ends the others (they would otherwise wait in the rendezvous
    # or the gather until the backend's timeout)
    while any(p.poll() is None for p in procs):
        if any(p.poll() not in (None, 0) for p in procs):
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    p.kill()
            break
        time.sleep(0.05)
    reader.join(timeout=30)
    rcs = [p.wait() for p in procs]
    sys.stdout.write(out[0] if out else "")
    sys.stdout.flush()
    bad = [rc for rc in rcs if rc != 0]
    return bad[0] if bad else 0


def world_from_env(a):
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return rank, world, local


# ----------------------------------------------------------------------------- CPU baseline
def cpu_info() -> dict:
    model = ""
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count() or 1
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return {"model": model, "nproc": os.cpu_count(), "affinity": usable,
            # the GPU box grants one GPU's job a CPU share (OMP_NUM_THREADS there); all usable cores otherwise
            "threads": min(usable, omp) if omp > 0 else usable}


def _timed(fn, n0: int, total: int, budget: float):
    """Run fn(n) on growing prefixes until one run takes >= budget/4 s or the whole sample ran."""
    n = min(n0, total)
    while True:
        t0 = time.perf_counter()
        res = fn(n)
        dt = time.perf_counter() - t0
        if dt > budget / 4 or n >= total:
            return n, dt, res
        n = min(total, int(n * max(2.0, budget / 4 / max(dt, 1e-3))))


def _parity(du0_gpu, it_gpu, x_ref, it_ref, st_ref) -> dict:
    """The device's applied moves against the oracle's on the CPU sample (the checker's role)."""
    ok = st_ref == 1
    scale = np.maximum(1.0, np.abs(x_ref).max(axis=1))
    d = np.abs(du0_gpu - np.where(ok, x_ref[:, 0], 0.0))
    return {"qps": int(len(du0_gpu)), "schedule_match": float(np.mean(it_gpu == it_ref)),
            "max_abs_du0": float(d.max()), "max_rel_du0": float((d / scale).max())}


def cpu_baseline(kind: str, run, n0: int, total: int, budget: float, threads: int, what: str,
                 per_unit: int = 1):
    """Time the oracle (`run(n, nthreads)`) single-threaded and on `threads` OpenMP threads over a
    bounded prefix of the same batch (n units of `per_unit` QP solves each); returns the record and
    the multi-threaded run's results."""
    info = cpu_info()
    thr = threads or info["threads"]
    n1, dt1, _ = _timed(lambda n: run(n, 1), max(1 if per_unit > 1 else 8, n0 // 16), total, budget / 2)
    n, dt, res = _timed(lambda n: run(n, thr), n0, total, budget / 2)
    unit = "QPs" if per_unit == 1 else f"plants x {per_unit} steps"
    rec = {"value": n * per_unit / dt, "unit": "QP/s", "cores": thr, "kind": kind,
           "single_thread": {"value": n1 * per_unit / dt1, "sample": f"{n1} {unit}, {dt1:.2f} s"},
           "cpu": info,
           "sample": f"{n} {unit} of the batch (its first {n}): {what}, fp64, OpenMP {thr} threads, {dt:.2f} s"}
    return rec, n, res


# ----------------------------------------------------------------------------- config 4
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
        return mdist.gather_moves(dist, U_d, world, rank, gathered)

    wall, got = _timed_loop(a, step, dist, world, dev)
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
        return None
    tf = lambda f, ms: f / (ms * 1e-3) / 1e12  # noqa: E731
    peak = PEAK_TFLOPS["f64"]
    rec = _header(a, world, B * world * a.steps / wall, wall, "f64",
                  "QP solves/sec (quad-rotor n_x=12, n_u=4, N=30 batch)",
                  "synthetic (hover linearisations, mass/inertia +-10% counter-based per plant; X ~ N(0, diag), U ~ U(-w0/2, w0/2))",
                  {"workload": f"cfg4: {B} quad-rotor plants per GPU (n_x {nx}, n_u {nu}, n_y {ny}), N={N} "
                               f"(n={n}, m={2 * n}): on-device MIMO condensing + setup + one controllerStep each",
                   "batch_per_gpu": B, "horizon": N, "parallelism": f"dp{world}"})
    rec.update({
        # dominant stage: the per-QP solve (Gauss-Jordan KKT inverse + ADMM iterations, fp64 VALU)
        "roofline": {"bound": "valu", "achieved": tf(solve_flops, solve_ms), "peak": peak, "unit": "TFLOP/s",
                     "frac": tf(solve_flops, solve_ms) / peak, "traffic": traffic_per_solve("quadrotor_f64", B, N),
                     "kernel": "mimo_solve_kernel (fp64 vector peak)", "kernel_ms": solve_ms,
                     "flops_per_step": solve_flops,
                     "flops_note": "algorithmic for the structured solve: 2n^3 per KKT inverse (1 + one per QP whose "
                                   "rho adapted), iters x (2n^2 + structured A products + 30n) "
                                   "(workload.flops_mimo_solve)"},
        "stages": {"setup_ms": setup_ms, "solve_ms": solve_ms, "step_ms": kern_ms,
                   "setup_roofline": {"bound": "valu", "achieved": tf(setup_flops, setup_ms), "peak": peak,
                                      "unit": "TFLOP/s", "frac": tf(setup_flops, setup_ms) / peak,
                                      "traffic": traffic_per_solve("quadrotor_setup_f64", B, N),
                                      "kernel": "mimo_setup_kernel", "flops_per_step": setup_flops,
                                      "note": "timed span includes the host read-back of the setup status word"}},
        "dense_equivalent": {"flops_per_step": dense, "achieved": tf(dense, kern_ms), "frac": tf(dense, kern_ms) / peak,
                             "note": "SURVEY §8d count: dense condensing + Ruiz + one KKT LDL + iters x F_iter(n, m)"},
        "iters": {"mean": float(iters.mean()), "max": int(iters.max()),
                  "solved_frac": float(np.mean(status == sm.SOLVED)), "rho_adapted_frac": float(np.mean(fact > 1))},
        "collective": _collective(dist, world, got),
    })
    if a.cpu_seconds > 0 and world == 1:  # (rank 0 at N = 1 only)
        import oracle

        run = lambda n, t: oracle.mimo_plants_step(sh, Ad[:n], Bd[:n], X[:n], U[:n], N, nthreads=t)  # noqa: E731
        rec["cpu_baseline"], ns, (U_ref, x_ref, st_ref, it_ref) = cpu_baseline(
            "port", run, 64, B, a.cpu_seconds, a.cpu_threads,
            "oracle/mpc_mimo.c condense + osqp_dense.c setup + one controllerStep per plant")
        du = U_d[:ns].cpu().numpy() - U[:ns]
        rec["parity"] = _parity(du[:, 0], iters[:ns], x_ref, it_ref, st_ref)
    return rec


# ----------------------------------------------------------------------------- shared pieces
def _header(a, world, value, wall, dtype, metric, data, config):
    return {"metric": metric, "value": value, "unit": "QP/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": wall / a.steps * 1e3, "higher_is_better": True,
            "scaling": getattr(a, "scaling", "weak"), "vs_baseline": None, "dtype": dtype, "data": data,
            "config": config}


def blocks(a, rank, world):
    """This rank's block of the global counter-based stream: (start, count, padded length, QPs of the job).
    weak: --batch per rank; strong: --global-batch split into near-equal contiguous blocks, each rank's
    moves padded to the longest block for the equal-size gather."""
    from solvempc_amd import dist as mdist

    if a.scaling == "strong":
        start, count = mdist.strong_block(a.global_batch, rank, world)
        return start, count, -(-a.global_batch // world), a.global_batch
    start, count = mdist.weak_block(a.batch, rank)
    return start, count, count, a.batch * world


def _collective(dist, world, got):
    """What the gather saw: the process group's world size and how many moves reached rank 0."""
    if world == 1:
        return {"backend": None, "world_size": 1, "gathered": int(got[0].numel())}
    return {"backend": dist.get_backend(), "world_size": dist.get_world_size(),
            "gathered": int(sum(t.numel() for t in got))}


def _timed_loop(a, step, dist, world, dev):
    """W untimed warmup steps, then K timed steps between barrier + synchronize; max over ranks."""
    import torch

    sync = (lambda: torch.cuda.synchronize()) if dev.type == "cuda" else (lambda: None)  # noqa: E731
    for _ in range(a.warmup):
        step()
    sync()
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    got = None
    for i in range(a.steps):
        got = step(i)
    sync()
    if world > 1:
        dist.barrier()
    sync()
    wall = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([wall], device=dev if a.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall = float(t.item())
    return wall, got


def traffic_per_solve(name, batch, N):
    """HBM bytes of one bench step of the dominant kernel from the committed PMC pass of the same bench
    command (tools/gpu.sh pmc:<workload>,<dtype> -> tools/pmc_traffic.py -> profiles/pmc_traffic_<name>.json),
    or None when no pass of this batch and horizon is committed."""
    f = ROOT / "profiles" / f"pmc_traffic_{name}.json"
    try:
        d = json.loads(f.read_text())
    except (OSError, ValueError):
        return None
    if d.get("batch") != batch or d.get("horizon") != N:
        return None
    return d.get("bytes_per_solve")


def mfma_util(dtype, kernel="admm_tile_kernel"):
    """MFMA utilisation of the dominant kernel from the committed PMC pass (tools/pmc.sh +
    tools/pmc_mfma.py -> profiles/pmc_mfma_<dtype>.json: SQ_VALU_MFMA_BUSY_CYCLES over SIMD-cycles), or
    None.  A recorded measurement of the same bench command, not re-measured by this run."""
    f = ROOT / "profiles" / f"pmc_mfma_{dtype}.json"
    try:
        d = json.loads(f.read_text()).get(kernel, {})
    except (OSError, ValueError):
        return None
    if "mfma_util" not in d:
        return None
    return {"value": d["mfma_util"], "source": f"profiles/{f.name} (rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES, "
                                              f"GRBM_GUI_ACTIVE; bench.py --steps 3 --warmup 1)"}


def main_dry(a, rank, world, dist):
    """--dry-run: the launcher, the rendezvous and the per-step gather of the applied moves on the
    CPU (gloo), no device work.  value is null: nothing is solved."""
    import torch

    from solvempc_amd import dist as mdist
    from solvempc_amd import workload

    start, count, pad, total = blocks(a, rank, world)
    _, U = workload.mpc_states(a.seed, start, count)
    U_t = torch.zeros(pad, dtype=torch.float64)
    U_t[:count] = torch.from_numpy(U)
    pg = mdist.PipelinedGather(dist, world, rank, U_t.clone())  # (the bench's overlapped per-step gather)

    def step(i=None):
        pg.buffer().copy_(U_t)
        return pg.gather()

    wall, got = _timed_loop(a, step, dist, world, torch.device("cpu"))
    pg.finish()
    if rank != 0:
        return None
    rec = _header(a, world, None, wall, a.dtype, "QP solves/sec (n_x=4, n_u=1, N=20 batch)",
                  "dry run: no device, no solve", {"workload": "dry run of the launcher and the gather",
                                                    "batch_per_gpu": count, "global_batch": total,
                                                    "parallelism": f"dp{world}"})
    rec["dry_run"] = True
    rec["collective"] = _collective(dist, world, got)
    full = (mdist.unpad(got, total, world) if a.scaling == "strong" else torch.cat(got)).numpy()
    rec["collective"]["gathered"] = int(full.size)
    rec["collective"]["matches_stream"] = bool(np.array_equal(full, workload.mpc_states(a.seed, 0, total)[1]))
    return rec


def cfg3_block(r3: dict) -> dict:
    """The cfg2 line's `cfg3_strong` block: BASELINE config 3's job (one global batch of randomised plants split
    over the ranks, condense + setup + one controllerStep each, U gathered to rank 0) from its own record."""
    rl = r3.get("roofline") or {}
    keep = ("value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "scaling", "dtype", "config", "iters",
            "collective")
    out = {k: r3[k] for k in keep if k in r3}
    out["metric"] = "QP solves/sec (BASELINE config 3: 1 M randomised plants, n_x=4, n_u=1, N=20, sharded, RCCL gather)"
    if rl:
        out["roofline"] = {k: rl[k] for k in ("bound", "achieved", "peak", "unit", "frac", "kernel", "kernel_ms")
                           if k in rl}
        out["roofline"]["note"] = "rank 0's kernel time and plants (the ranks' blocks differ by at most one plant)"
    if r3.get("dry_run"):
        out["dry_run"] = True
    return out


# ----------------------------------------------------------------------------- main
def main():
    argv = sys.argv[1:]
    a = parse(argv)
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(a, argv))
    rank, world, local = world_from_env(a)
    if world != a.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {a.gpus}")
    import torch

    dist = None
    if world > 1:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if a.backend == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(a.backend, rank=rank, world_size=world)
    elif not a.dry_run:
        torch.cuda.set_device(local)
    try:
        if a.dry_run:
            rec = main_dry(a, rank, world, dist)
        elif a.workload == "quadrotor":
            rec = main_quadrotor(a, rank, world, local, dist, torch.device("cuda", local))
        else:
            rec = main_lti(a, rank, world, local, dist, torch.device("cuda", local))
        if a.workload == "cfg2" and a.cfg3_strong and a.scaling == "weak":
            # BASELINE config 3 as written, in the same run (and so in the driver's multi-GPU SCALE lines)
            a3 = parse(["--workload", "perplant", "--scaling", "strong", "--gpus", str(a.gpus),
                        "--global-batch", str(a.cfg3_global_batch), "--steps", str(a.steps),
                        "--warmup", str(min(a.warmup, 2)), "--cpu-seconds", "0", "--backend", a.backend])
            rec3 = (main_dry(a3, rank, world, dist) if a.dry_run
                    else main_lti(a3, rank, world, local, dist, torch.device("cuda", local)))
            if rank == 0:
                rec["cfg3_strong"] = cfg3_block(rec3)
        if rank == 0:
            print(json.dumps(rec))
    finally:
        if dist:
            dist.destroy_process_group()


def main_lti(a, rank, world, local, dist, dev):
    """Configs 2 (shared plant), 3 (per-plant condensing + setup + step) and 5 (stream)."""
    import torch

    import solvempc_amd as sm
    from solvempc_amd import dist as mdist
    from solvempc_amd import workload

    N = a.horizon
    start, B, pad, total = blocks(a, rank, world)  # this rank's QPs (weak: --batch each; strong: a block of the job)
    plant = workload.reference_plant()
    ops = sm.mpc.condense({"Ad": plant["Ad"][None], "Bd": plant["Bd"][None], "Cd": plant["Cd"][None],
                           "K": plant["K"][None], "Q": [plant["Q"]], "R": [plant["R"]], "RD": [plant["RD"]]},
                          N, device=local)
    ops = {k: v[0] for k, v in ops.items()}
    stream_mode = a.workload == "stream"
    perplant = a.workload == "perplant"
    X, U = workload.stream_states(a.seed, start, B) if stream_mode else workload.mpc_states(a.seed, start, B)
    l = np.full(2 * N, -np.finfo(np.float64).max)
    u0 = ops["W0"].copy()  # W0 + Sbar 0 + Ku 0 (:43)

    if perplant:  # config 3: every QP its own plant, condensed and set up on the device each step
        Ad, Bd = workload.randomized_plants(plant, a.seed, start, B)
        solver = sm.BatchSolver(N, 2 * N, B, B, a.dtype, local)
        tdev = lambda v: torch.as_tensor(np.ascontiguousarray(v, dtype=np.float64)).to(dev)  # noqa: E731
        plant_d = [tdev(Ad), tdev(Bd), tdev(np.tile(plant["Cd"], (B, 1))), tdev(np.tile(plant["K"], (B, 1))),
                   tdev(np.full(B, plant["Q"])), tdev(np.full(B, plant["R"])), tdev(np.full(B, plant["RD"]))]
    else:
        solver = sm.BatchSolver(N, 2 * N, B, 1, a.dtype, local)
        solver.setup(ops["P"], np.zeros(N), ops["A"], l, u0)
        solver.mpc_set_operators(ops["Fx"], ops["Fu"], ops["Fr"], ops["Sbar"], ops["Ku"], ops["W0"])
    X_d = torch.from_numpy(X).to(dev)
    U0_d = torch.zeros(pad, dtype=torch.float64, device=dev)  # (strong: padded to the longest block, gather)
    U0_d[:B] = torch.from_numpy(U).to(dev)
    U_d = U0_d.clone()
    stream = torch.cuda.current_stream(dev)
    sptr = stream.cuda_stream
    gathered = [torch.empty_like(U_d) for _ in range(world)] if rank == 0 else None
    # the per-step gather of the moves overlaps the next step (double-buffered U, async RCCL gather); the
    # stream workload (tens of ms per step) gathers in line
    pg = mdist.PipelinedGather(dist, world, rank, U_d) if not stream_mode else None
    U_line = U_d

    if stream_mode:
        solver.mpc_set_plant(plant["Ad"], plant["Bd"])
        side = torch.cuda.Stream(dev)  # graph capture needs a non-default stream
        stream, sptr = side, side.cuda_stream
        X0_d = X_d.clone()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
    cur = torch.cuda.current_stream(dev)

    def step(i=None):
        U_d = pg.buffer() if pg else U_line
        U_d.copy_(U0_d)          # every step: the reference's first control step of each plant
        if not perplant:         # (perplant: the setup inside the step resets the state)
            solver.reset_state()  # post-setup solver state (x = z = y = 0, rho = settings.rho)
        if stream_mode:
            X_d.copy_(X0_d)
            stream.wait_stream(cur)  # the resets above ran on the current stream
        if i is not None:
            ev[i][0].record(stream)
        if stream_mode:  # config 5: ctrl_steps warm-started control steps + plant updates (hipGraph)
            solver.mpc_run_device(X_d.data_ptr(), U_d.data_ptr(), plant["xref"], a.ctrl_steps, a.seed, start, 0,
                                  a.noise, sptr)
        else:
            if perplant:  # every plant's ctor + controllerStep in one pass, operators on chip
                solver.mpc_plants_step_device(4, 10, *[t.data_ptr() for t in plant_d], X_d.data_ptr(),
                                              U_d.data_ptr(), plant["xref"], sptr)
            else:
                solver.mpc_step_device(X_d.data_ptr(), U_d.data_ptr(), plant["xref"], sptr)
        if i is not None:
            ev[i][1].record(stream)
        if stream_mode:
            cur.wait_stream(stream)
            return mdist.gather_moves(dist, U_d, world, rank, gathered)
        return pg.gather()

    wall, got = _timed_loop(a, step, dist, world, dev)
    if pg:
        U_d = pg.finish()  # the last step's moves
    kern_ms = float(np.mean([s.elapsed_time(e) for s, e in ev]))
    U_out = U_d[:B].cpu().numpy().copy()  # this step's applied U (the parity block's device side)

    status, iters, rho_f = solver.info()
    # cfg2 at N = 1: the other precisions on the same batch with the same protocol (the `variants` block)
    variants = {}
    if a.workload == "cfg2" and a.variants and world == 1 and a.scaling == "weak":
        for vdt in [d for d in ("f32", "mixed", "f64") if d != a.dtype]:
            vs = sm.BatchSolver(N, 2 * N, B, 1, vdt, local)
            vs.setup(ops["P"], np.zeros(N), ops["A"], l, u0)
            vs.mpc_set_operators(ops["Fx"], ops["Fu"], ops["Fr"], ops["Sbar"], ops["Ku"], ops["W0"])
            vev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]

            def vstep(i=None, vs=vs, vev=vev):
                U_d.copy_(U0_d)
                vs.reset_state()
                if i is not None:
                    vev[i][0].record(stream)
                vs.mpc_step_device(X_d.data_ptr(), U_d.data_ptr(), plant["xref"], sptr)
                if i is not None:
                    vev[i][1].record(stream)
                return [U_d]

            vwall, _ = _timed_loop(a, vstep, dist, world, dev)
            vst, vit, _ = vs.info()
            vkind, vpaired = vs.path()
            vflops = float(workload.flops_per_qp(N, 2 * N, 4, vit, paired=vpaired).sum())
            vms = float(np.mean([s_.elapsed_time(e_) for s_, e_ in vev]))
            variants[vdt] = {"dtype": DTYPE_NAME[vdt], "value": B * a.steps / vwall, "ms_per_step": vwall / a.steps * 1e3,
                             "kernel_ms": vms, "achieved_tflops": vflops / (vms * 1e-3) / 1e12,
                             "iters_mean": float(vit.mean()), "solved_frac": float(np.mean(vst == sm.SOLVED)),
                             "_U": U_d[:B].cpu().numpy().copy(), "_it": vit}
            vs.close()
    kind, paired = solver.path()
    qps_per_step = total * (a.ctrl_steps if stream_mode else 1)  # every rank's QPs of one bench step
    if stream_mode:  # iterations every QP ran over all control steps of the last bench step (device counters)
        it_total = solver.stream_iterations()
        flops = float(workload.flops_per_qp_total(N, 2 * N, 4, it_total, a.ctrl_steps, paired=paired).sum())
        flops_dense = float(workload.flops_per_qp_total(N, 2 * N, 4, it_total, a.ctrl_steps).sum())
    else:
        flops = float(workload.flops_per_qp(N, 2 * N, 4, iters, paired=paired).sum())
        flops_dense = float(workload.flops_per_qp(N, 2 * N, 4, iters).sum())
    achieved = flops / (kern_ms * 1e-3) / 1e12
    solved = float(np.mean(status == sm.SOLVED))
    if rank != 0:
        return None
    total_qps = qps_per_step * a.steps / wall
    config = ({"workload": f"cfg2: {B} identical LTI plants per GPU, N={N} (n={N}, m={2 * N}), one controllerStep each",
               "batch_per_gpu": B, "horizon": N, "parallelism": f"dp{world}"} if a.workload == "cfg2" else
              {"workload": f"cfg3: {total} randomised plants (Ad, Bd +-2% ~ N(0,1), rho(Ad) < 1), {B} on rank 0, "
                           f"N={N}: on-device condensing + setup + one controllerStep each",
               "batch_per_gpu": B, "global_batch": total, "horizon": N, "parallelism": f"dp{world}"} if perplant else
              {"workload": f"cfg5: {B} plants per GPU x {a.ctrl_steps} warm-started control steps, simulated plant "
                           f"(noise std {a.noise}, X0 ~ N(0, {workload.STREAM_X_SCALE}^2 diag(.1,.1,.05,.5)), U0 = 0), "
                           f"one launch for all steps (tile stream mode where the shape allows), N={N}",
               "batch_per_gpu": B, "horizon": N, "ctrl_steps": a.ctrl_steps, "parallelism": f"dp{world}"})
    peak = PEAK_TFLOPS.get(a.dtype)
    split = None
    if a.dtype == "mixed":
        if kind == "tile" and not stream_mode and not perplant:
            f64s, f32s = workload.flops_split_mixed(N, 2 * N, 4, iters, sm.MPCQ_MIX_R, paired=paired)
            split = (float(f64s.sum()), float(f32s.sum()))
        elif stream_mode and solver.stream_path() == "tile":  # (the tile stream mode runs the mixed loop)
            f64s, f32s = workload.flops_split_mixed_total(N, 2 * N, 4, it_total, a.ctrl_steps, sm.MPCQ_MIX_R,
                                                          paired=paired)
            split = (float(f64s.sum()), float(f32s.sum()))
        if split:
            peak = (split[0] + split[1]) / (split[0] / PEAK_TFLOPS["f64"] + split[1] / PEAK_TFLOPS["f32"])
        else:  # (every other path runs MPCQ_F64_MIXED in fp64)
            peak = PEAK_TFLOPS["f64"]
    rec = _header(a, world, total_qps, wall, DTYPE_NAME[a.dtype], "QP solves/sec (n_x=4, n_u=1, N=20 batch)",
                  "synthetic (counter-based X ~ N(0, diag(.1,.1,.05,.5)), U ~ U(-1,1); reference plant config)"
                  if not stream_mode else "synthetic (counter-based initial states and plant noise; reference plant config)",
                  config)
    rec["roofline"] = {
        "bound": "mfma", "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
        "frac": achieved / peak,
        "traffic": traffic_per_solve(a.dtype if not stream_mode else f"stream_{a.dtype}", B, N),
        "mfma_util": mfma_util(a.dtype) if a.workload == "cfg2" and B == 65536 else None,
        "kernel": ({"tile": "admm_tile_kernel, stream mode (one launch: every plant's control steps and "
                            "plant updates, one plant per MFMA column)",
                    "wave": "stream_wave_kernel (one launch: every control step and plant update)",
                    "graph": f"admm_{kind}_kernel (per-step launches, hipGraph)"}[solver.stream_path()]
                   if stream_mode else
                   f"admm_{kind}_kernel{' (paired loop)' if paired else ''} (all launches of "
                   f"{'the step' if not stream_mode else 'the control steps'})"),
        "kernel_ms": kern_ms, "flops_per_step": flops,
        "dense_equivalent": {"flops_per_step": flops_dense, "achieved": flops_dense / (kern_ms * 1e-3) / 1e12,
                             "frac": flops_dense / (kern_ms * 1e-3) / 1e12 / peak},
        "flops_note": "algorithmic: sum over QPs of iters*F_iter + checks*F_check + front end (SURVEY §8d, DESIGN §4.1), "
                      "actual per-QP iteration counts"
                      + ("; F_iter and F_check count the m/2-row products the paired loop performs "
                         "(dense_equivalent: the dense 4nm count)" if paired else "")
                      + ("; stream: every control step's iterations, accumulated on the device" if stream_mode else "")}
    if split:
        rec["roofline"]["peak_note"] = (f"mixed: {split[0] / sum(split):.3f} of the FLOPs in fp64 (the last {sm.MPCQ_MIX_R} "
                                        f"iterations of every check interval, the checks, the front end), the rest "
                                        f"fp32; peak = the matrix cores' rate for that split "
                                        f"(f64 {PEAK_TFLOPS['f64']}, f32 {PEAK_TFLOPS['f32']} TF)")
    rec["iters"] = {"mean": float(iters.mean()), "max": int(iters.max()), "solved_frac": solved}
    if stream_mode:
        rec["iters"]["stream_total_mean"] = float(it_total.mean())
        rec["iters"]["stream_unsolved_steps"] = int(solver.stream_unsolved())
        rec["iters"]["final_max_abs_X"] = float(X_d.abs().max().item())
    rec["collective"] = _collective(dist, world, got)
    if a.scaling == "strong":  # (the blocks are padded to the longest for the equal-size gather)
        rec["collective"]["gathered"] = int(mdist.unpad(got, total, world).numel()) if world > 1 else B
    if perplant:
        # One kernel per step: condensing + Ruiz + KKT inverse (fp64) and the ADMM (T = dtype) of every
        # plant, two plants per wave.  FLOPs as the kernel performs them (workload.flops_plant_step;
        # a refactorisation per plant whose rho moved), priced at the vector peak of the ADMM's type.
        rho0 = solver.settings.rho if a.dtype != "f32" else float(np.float32(solver.settings.rho))
        refac = (rho_f != rho0).astype(np.float64)
        merged = a.dtype != "f32"  # (the fp64 kernel's one-GEMV iteration, mpcq_plant.hip)
        pf = float(workload.flops_plant_step(N, 4, iters, refac, solver.settings.scaling, merged=merged).sum())
        ach = pf / (kern_ms * 1e-3) / 1e12
        rec["roofline"] = {"bound": "valu", "achieved": ach, "peak": peak, "unit": "TFLOP/s",
                           "frac": ach / peak, "traffic": traffic_per_solve(f"perplant_{a.dtype}", B, N),
                           "kernel": "plant_step_kernel (condense + setup + solve, one pass)", "kernel_ms": kern_ms,
                           "flops_per_step": pf,
                           "flops_note": "as performed (workload.flops_plant_step): condensing by lag scans, Ruiz, "
                                         + ("2N^3 + 6N^2 per KKT inverse (setup + one per rho change), 2N^2 + 28N per "
                                            "iteration (one GEMV, A^'w and A^x by suffix / prefix scans)" if merged else
                                            "2N^3 + 10N^2 per KKT inverse (setup + one per rho change), 4N^2 + 23N per "
                                            "iteration (A structural: prefix / suffix scans)")
                                         + ", 2N^2 + 36N per check; the fp64 setup is priced at the same peak",
                           "dense_equivalent": {"flops_per_step": flops_dense + B * workload.flops_plant_setup(N, 2 * N),
                                                "note": "SURVEY §8d: dense F_iter / F_check + F_condense + Ruiz + one LDL"}}
        rec["iters"]["rho_adapted_frac"] = float(refac.mean())
    if a.cpu_seconds > 0 and stream_mode and world == 1:  # (rank 0 at N = 1 only)
        import oracle

        run = lambda n, t: oracle.stream_run(plant, X[:n], U[:n], N, a.ctrl_steps, a.seed, start, 0, a.noise,  # noqa: E731
                                             xref=plant["xref"], nthreads=t)
        rec["cpu_baseline"], ns, (Xc, Uc, itc, unc) = cpu_baseline(
            "port", run, 16, B, a.cpu_seconds, a.cpu_threads,
            "oracle/mpc_batch.c ora_stream_run (one warm-started OSQP-0.6 restatement per plant, the device's "
            "noise stream)", per_unit=a.ctrl_steps)
        # the device's last bench step on the same plants (informational: fp32 and fp64 closed loops
        # drift apart by rounding over the steps, each step's parity is tests/test_gpu.py's)
        rec["parity"] = {"plants": int(ns), "steps": a.ctrl_steps,
                         "it_total_match": float(np.mean(it_total[:ns] == itc)),
                         "it_total_rel_diff": float(np.abs(it_total[:ns] - itc).sum() / max(1, itc.sum())),
                         "max_abs_dU_final": float(np.abs(U_out[:ns] - Uc).max()),
                         "unsolved_steps_cpu": int(unc.sum())}
    if a.cpu_seconds > 0 and not stream_mode and world == 1:  # (rank 0 at N = 1 only)
        import oracle

        if perplant:
            run = lambda n, t: oracle.plants_step(plant, Ad[:n], Bd[:n], X[:n], U[:n], N, nthreads=t)  # noqa: E731
            rec["cpu_baseline"], ns, (U_ref, st_ref, it_ref) = cpu_baseline(
                "port", run, 256, B, a.cpu_seconds, a.cpu_threads,
                "oracle/mpc_batch.c condense + osqp_dense.c setup + one controllerStep per plant")
            x_ref = (U_ref - U[:ns])[:, None]
        else:
            q0 = np.zeros(N)
            q, u = oracle.gradient(ops, X, U), oracle.upper_bound(ops, X, U)
            run = lambda n, t: oracle.batch_solve(ops["P"], ops["A"], q0, l, u0, q[:n], u[:n], nthreads=t)  # noqa: E731
            rec["cpu_baseline"], ns, (x_ref, st_ref, it_ref, _) = cpu_baseline(
                "port", run, 256, B, a.cpu_seconds, a.cpu_threads, "oracle/osqp_dense.c (OSQP-0.6 restatement)")
        du = U_out[:ns] - U[:ns]
        rec["parity"] = _parity(du, iters[:ns], x_ref, it_ref, st_ref)
        if perplant:
            rec["parity"].pop("max_rel_du0")  # (the per-plant oracle returns U only)
        for v in variants.values():
            v["parity"] = _parity(v["_U"][:ns] - U[:ns], v["_it"][:ns], x_ref, it_ref, st_ref)
    if variants:
        for v in variants.values():
            v.pop("_U")
            v.pop("_it")
        rec["variants"] = variants
    return rec


if __name__ == "__main__":
    main()
