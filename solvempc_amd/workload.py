"""Synthetic LTI-MPC workloads (BASELINE.json configs), counter-based so every rank can generate its
own shard of a global batch without communication and results are shard-invariant.

Random numbers: SplitMix64 of (seed, global QP index, draw index) -> uniform (0,1) doubles;
normals by Box-Muller.  The reference has no data source other than a serial port
(src/SerialPort.cpp), so the states are synthetic by construction.
"""
from __future__ import annotations

import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)
X_STD = np.sqrt([0.1, 0.1, 0.05, 0.5])  # X ~ N(0, diag(.1,.1,.05,.5))


def _splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def uniforms(seed: int, start: int, count: int, draws: int, draw0: int = 0, idx=None) -> np.ndarray:
    """(count, draws) uniforms in (0, 1) for global QP indices start .. start+count-1 (or the index
    array `idx`; draw indices draw0 .. draw0+draws-1; mpcq_stream.hip's device generator is the same
    function)."""
    idx = (np.arange(start, start + count, dtype=np.uint64) if idx is None
           else np.asarray(idx, dtype=np.uint64))[:, None]
    d = np.arange(draw0, draw0 + draws, dtype=np.uint64)[None, :]
    with np.errstate(over="ignore"):
        key = _splitmix64(np.uint64(seed) * np.uint64(0x632BE59BD9B4E019) + np.uint64(1))
        x = _splitmix64(key ^ (idx * np.uint64(0x100000001B3) + d * np.uint64(0xD6E8FEB86659FD93)))
    return ((x >> np.uint64(11)).astype(np.float64) + 0.5) * (1.0 / 9007199254740992.0)


def normals(seed: int, start: int, count: int, k: int) -> np.ndarray:
    u = uniforms(seed, start, count, 2 * ((k + 1) // 2))
    r = np.sqrt(-2.0 * np.log(u[:, 0::2]))
    th = 2.0 * np.pi * u[:, 1::2]
    z = np.concatenate([r * np.cos(th), r * np.sin(th)], axis=1)
    return z[:, :k]


def plant_noise(seed: int, start: int, count: int, step: int, nx: int, std: float) -> np.ndarray:
    """w of the simulated plant at control step `step` (mpcq_stream.hip simulate_kernel): Box-Muller
    pairs from draws step*64 + 2p, 2p+1; component t = r_t cos(th_t) for t < ceil(nx/2), else the sine
    of pair t - ceil(nx/2)."""
    npairs = (nx + 1) // 2
    u = uniforms(seed, start, count, 2 * npairs, draw0=64 * step)
    r = np.sqrt(-2.0 * np.log(u[:, 0::2]))
    th = 2.0 * np.pi * u[:, 1::2]
    z = np.concatenate([r * np.cos(th), r * np.sin(th)], axis=1)[:, :nx]
    return std * z


def simulate(Ad, Bd, X, U, w) -> np.ndarray:
    """X <- Ad X + Bd U + w for a batch (shared plant)."""
    return X @ np.asarray(Ad).T + np.asarray(U)[:, None] * np.asarray(Bd)[None, :] + w


def mpc_states(seed: int, start: int, count: int, u_range: float = 1.0):
    """Config 2 states: X ~ N(0, diag(.1,.1,.05,.5)), U ~ U(-u_range, u_range) (0 when u_range=0)."""
    X = normals(seed, start, count, 4) * X_STD
    U = (2.0 * uniforms(seed ^ 0x5A5A, start, count, 1)[:, 0] - 1.0) * u_range
    return X, U


# Config 5 (receding-horizon stream) starts inside the reference controller's region of attraction.
# The config-2 law above puts |K X| ~ 1,200 on the inner loop's PWM command (K = [-50, -150, 5500,
# 350], K X = -(PWM) + K0 U with |PWM| <= 255 the constraint rows of ModelPredictiveControlAPI.cpp:
# 335,364-368): the actuator saturates from the first step and the cart-pole's open-loop pole
# (|lambda| = 1.0797 in Ad + Bd K / K0) diverges whatever the QP returns (measured with the oracle:
# x1.08 per step).  A tenth of that spread (|K X| ~ 120) with the reference's own initial input
# U = 0 (:23) keeps every plant SOLVED and bounded over 1,000 steps at noise std 1e-2.
STREAM_X_SCALE = 0.1


def stream_states(seed: int, start: int, count: int):
    """Config 5 initial states: X ~ N(0, STREAM_X_SCALE^2 diag(.1,.1,.05,.5)), U = 0."""
    X = normals(seed, start, count, 4) * (X_STD * STREAM_X_SCALE)
    return X, np.zeros(count)


def randomized_plants(plant: dict, seed: int, start: int, count: int, rel: float = 0.02, attempts: int = 64):
    """Config 3 plants for global indices start .. start+count-1: Ad = Ad0 o (1 + rel eps),
    Bd = Bd0 o (1 + rel eps), eps ~ N(0, 1) (Box-Muller on draws 32a .. 32a+19 of attempt a); a draw
    with spectral radius rho(Ad) >= 1 is rejected and redrawn (after `attempts` the nominal plant).
    A plant depends on its global index only, so large batches run as index blocks on a thread pool
    (numpy and LAPACK release the GIL): the same arrays as one block."""
    import os
    from concurrent.futures import ThreadPoolExecutor

    workers = min(16, os.cpu_count() or 1, max(1, count // 16384))
    if workers <= 1:
        return _randomized_block(plant, seed, start, count, rel, attempts)
    base, rem = divmod(count, workers)
    blocks = [(start + w * base + min(w, rem), base + (1 if w < rem else 0)) for w in range(workers)]
    with ThreadPoolExecutor(workers) as ex:
        parts = list(ex.map(lambda b: _randomized_block(plant, seed, b[0], b[1], rel, attempts), blocks))
    return np.concatenate([p_[0] for p_ in parts]), np.concatenate([p_[1] for p_ in parts])


def _randomized_block(plant: dict, seed: int, start: int, count: int, rel: float, attempts: int):
    Ad0, Bd0 = np.asarray(plant["Ad"], dtype=np.float64), np.asarray(plant["Bd"], dtype=np.float64)
    nx = Ad0.shape[0]
    k = nx * nx + nx
    Ad = np.broadcast_to(Ad0, (count, nx, nx)).copy()
    Bd = np.broadcast_to(Bd0, (count, nx)).copy()
    todo = np.arange(count)
    for a in range(attempts):
        if todo.size == 0:
            break
        u = uniforms(seed, 0, 0, 2 * ((k + 1) // 2), draw0=32 * a, idx=start + todo)
        r = np.sqrt(-2.0 * np.log(u[:, 0::2]))
        th = 2.0 * np.pi * u[:, 1::2]
        eps = np.concatenate([r * np.cos(th), r * np.sin(th)], axis=1)[:, :k]
        cA = Ad0[None] * (1 + rel * eps[:, :nx * nx].reshape(-1, nx, nx))
        cB = Bd0[None] * (1 + rel * eps[:, nx * nx:])
        ok = np.abs(np.linalg.eigvals(cA)).max(axis=1) < 1.0
        Ad[todo[ok]], Bd[todo[ok]] = cA[ok], cB[ok]
        todo = todo[~ok]
    return Ad, Bd


def shard(total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous block [start, start+count) of a global index range for one rank."""
    base, rem = divmod(total, world)
    start = rank * base + min(rank, rem)
    return start, base + (1 if rank < rem else 0)


def reference_plant(path=None) -> dict:
    """The reference plant/weights (config/MPC_API.json values, committed as tests/golden data)."""
    import json
    from pathlib import Path

    p = Path(path) if path else Path(__file__).resolve().parent.parent / "tests" / "golden" / "plant_mpc_api.json"
    cfg = json.loads(p.read_text())
    return {
        "Ad": np.asarray(cfg["Ad"], dtype=np.float64).reshape(4, 4),
        "Bd": np.asarray(cfg["Bd"], dtype=np.float64).reshape(4),
        "Cd": np.asarray(cfg["Cd"], dtype=np.float64).reshape(4),
        "K": np.asarray(cfg["K"], dtype=np.float64).reshape(4),
        "Q": float(np.asarray(cfg["Q"]).reshape(-1)[0]),
        "R": float(np.asarray(cfg["R"]).reshape(-1)[0]),
        "RD": float(np.asarray(cfg["RD"]).reshape(-1)[0]),
        "xref": float(cfg.get("xref", 0.0)),
    }


def flops_per_qp(n: int, m: int, nx: int, iters: np.ndarray, check: int = 25, paired: bool = False) -> np.ndarray:
    """Algorithmic FLOPs of one solve: iters*F_iter + checks*F_check + front end.
    F_iter = 4nm + 2n^2 + 9m + 6n; F_check = 4nm + 2n^2 + 6m + 4n; front end (q, u, W'q^)
    = 2n(nx+1+n) + 2m(nx+1) + 2n^2.  No refactorisation FLOPs: rho updates are diagonal.
    paired: the tile kernel's paired loop (rows n + j of A = -rows j) performs every A product (B'w,
    B eta, and A x, A'y of the check iterations) over the m/2 distinct rows: F_iter = 2nm + 2n^2 +
    9m + 6n, F_check = 2nm + 2n^2 + 6m + 4n (the reduced counts it performs; SURVEY §8d asks for
    them when the A structure is exploited)."""
    it = np.asarray(iters, dtype=np.float64)
    f_iter, f_check, f_front = _flop_terms(n, m, nx, paired)
    return it * f_iter + np.floor(it / check) * f_check + f_front


def flops_split_mixed(n: int, m: int, nx: int, iters: np.ndarray, mix_r: int, check: int = 25,
                      paired: bool = False) -> tuple[np.ndarray, np.ndarray]:
    """flops_per_qp of an MPCQ_F64_MIXED solve split by the arithmetic that performs it: (fp64, fp32).
    Iteration i (1-based) runs in fp64 when (i - 1) % check >= check - mix_r (the last mix_r of every
    check interval: the fp32 stretch's damping and the info iteration), in fp32 otherwise; the check
    products and the front end are fp64."""
    it = np.asarray(iters, dtype=np.int64)
    f_iter, f_check, f_front = _flop_terms(n, m, nx, paired)
    r = min(max(int(mix_r), 1), check)
    full, rem = it // check, it % check
    n64 = full * r + np.maximum(rem - (check - r), 0)
    f64 = n64 * float(f_iter) + full * float(f_check) + f_front
    f32 = (it - n64) * float(f_iter)
    return f64.astype(np.float64), f32.astype(np.float64)


def _flop_terms(n: int, m: int, nx: int, paired: bool):
    rows = m // 2 if paired else m  # the paired loop's A products run over the m/2 distinct rows
    f_iter = 4 * n * rows + 2 * n * n + 9 * m + 6 * n
    f_check = 4 * n * rows + 2 * n * n + 6 * m + 4 * n
    f_front = 2 * n * (nx + 1 + n) + 2 * m * (nx + 1) + 2 * n * n
    return f_iter, f_check, f_front


def flops_per_qp_total(n: int, m: int, nx: int, iters_total, solves: int, check: int = 25,
                       paired: bool = False) -> np.ndarray:
    """flops_per_qp over `solves` warm-started solves of each QP from the device's per-QP total of
    iterations (mpcq_mpc_stream_counters); checks counted as floor(total / check) (every solve of
    the stream stops on a check iteration, so this is exact when none hits max_iter)."""
    it = np.asarray(iters_total, dtype=np.float64)
    f_iter, f_check, f_front = _flop_terms(n, m, nx, paired)
    return it * f_iter + np.floor(it / check) * f_check + solves * f_front


def flops_split_mixed_total(n: int, m: int, nx: int, iters_total, solves: int, mix_r: int, check: int = 25,
                            paired: bool = False) -> tuple[np.ndarray, np.ndarray]:
    """flops_per_qp_total of an MPCQ_F64_MIXED stream split into (fp64, fp32): every solve of the stream
    stops on a check iteration, so each of its floor(total / check) intervals runs mix_r iterations
    (the last ones: damping and the info iteration) and its check in fp64, the rest in fp32; the front
    ends are fp64."""
    it = np.asarray(iters_total, dtype=np.int64)
    f_iter, f_check, f_front = _flop_terms(n, m, nx, paired)
    r = min(max(int(mix_r), 1), check)
    full = it // check
    n64 = full * r + np.maximum(it % check - (check - r), 0)
    f64 = n64 * float(f_iter) + full * float(f_check) + solves * float(f_front)
    f32 = (it - n64) * float(f_iter)
    return f64.astype(np.float64), f32.astype(np.float64)


def flops_plant_setup(n: int, m: int, N: int | None = None) -> float:
    """Algorithmic FLOPs of one plant's condensing + setup: F_condense (SISO)
    4N^3 + 10N^2 + 128N, Ruiz 10*3(n^2 + nm), F_setup 2n^2 m + n^3/3 + n^2 (one LDL of the KKT
    system; the eigen-basis setup does more work than this and is not credited for it)."""
    N = n if N is None else N
    return (4 * N ** 3 + 10 * N ** 2 + 128 * N) + 30 * (n * n + n * m) + (2 * n * n * m + n ** 3 / 3 + n * n)


def flops_plant_step(N: int, nx: int, iters, refactors, scaling: int = 10, check: int = 25,
                     merged: bool = False) -> np.ndarray:
    """FLOPs plant_step_kernel performs per plant (mpcq_plant.hip; FMA = 2, m = 2N with the paired rows,
    A = [K0 L; -K0 L] applied structurally):
    * condensing: the Ad^k Bd / Cd Ad^k recurrences 4 N nx^2, CAB and the free response 4 N nx, the
      per-lag products and prefix scans of the Hessian 2 N^2, P rows and q ~4 N^2;
    * Ruiz, `scaling` passes: P's row norms and scaling ~4 N^2, the structural A norms (scans) ~4 N;
    * per factorisation (setup + every refactorisation): M(rho) ~4 N^2, Gauss-Jordan 2 N^3, g = -M^-1 q
      2 N^2, the (A^ M^-1) columns by prefix sums 4 N^2;
    * front end 2 N (nx + 2);
    * per iteration: sigma M^-1 x and (A^ M^-1)' w, 4 N^2, the A^ x~ prefix scan ~3 N, ~20 N element-wise;
    * per check: P^ x 2 N^2, the A^ x and A^'y scans ~6 N, ~30 N of residuals and norms (fp64).
    merged (the fp64 kernel): one GEMV per iteration, M^-1 (sigma x + A^'w) with A^'w a suffix scan: 2 N^2
    + ~28 N per iteration, and no (A^ M^-1) columns per factorisation."""
    it = np.asarray(iters, dtype=np.float64)
    cond = 4 * N * nx * nx + 4 * N * nx + 6 * N * N
    ruiz = scaling * (4 * N * N + 4 * N)
    kkt = 2 * N ** 3 + (6 if merged else 10) * N * N
    per_it = 2 * N * N + 28 * N if merged else 4 * N * N + 23 * N
    return (cond + ruiz + 2 * N * (nx + 2) + (1 + np.asarray(refactors, dtype=np.float64)) * kkt
            + it * per_it + np.floor(it / check) * (2 * N * N + 36 * N))


# ----------------------------------------------------------------------------- config 4: quad-rotor
QUAD = {  # hover linearisation of a small quad-rotor (BASELINE config 4: n_x 12, n_u 4, N 30, dt 0.02)
    "mass": 0.5, "inertia": (2.3e-3, 2.3e-3, 4.0e-3), "g": 9.81, "dt": 0.02, "spread": 0.10,
    # outputs y = x (Cd = I); weights: position 10, attitude 1, velocity 1, body rates 0.1
    "q_diag": (10.0, 10.0, 10.0, 1.0, 1.0, 1.0, 1.0, 1.0, 1.0, 0.1, 0.1, 0.1),
    "r_diag": (0.1, 10.0, 10.0, 10.0), "rd_diag": (1.0, 100.0, 100.0, 100.0),
    # input box |u_k| <= w0 around hover: thrust deviation [N], roll/pitch/yaw torque [N m]
    "w0": (2.0, 0.05, 0.05, 0.02),
}
# State X ~ N(0, diag(s^2)): position 0.3 m, attitude 0.1 rad, velocity 0.3 m/s, rates 0.3 rad/s;
# the applied input U ~ U(-w0/2, w0/2).
QUAD_X_STD = np.array([0.3, 0.3, 0.3, 0.1, 0.1, 0.1, 0.3, 0.3, 0.3, 0.3, 0.3, 0.3])


def quadrotor_continuous(mass: float, Ixx: float, Iyy: float, Izz: float, g: float = 9.81):
    """Hover linearisation, x = [p (3), (phi, theta, psi), v (3), body rates (3)], u = [thrust deviation,
    tau_phi, tau_theta, tau_psi]: p' = v, angles' = rates, vx' = g theta, vy' = -g phi, vz' = T / m,
    rates' = tau / I."""
    A = np.zeros((12, 12))
    A[0, 6] = A[1, 7] = A[2, 8] = 1.0
    A[3, 9] = A[4, 10] = A[5, 11] = 1.0
    A[6, 4] = g
    A[7, 3] = -g
    B = np.zeros((12, 4))
    B[8, 0] = 1.0 / mass
    B[9, 1], B[10, 2], B[11, 3] = 1.0 / Ixx, 1.0 / Iyy, 1.0 / Izz
    return A, B


def zoh(A, B, dt: float):
    """Exact zero-order-hold discretisation: exp([[A, B], [0, 0]] dt) by its Taylor series (the
    augmented hover matrix is nilpotent, so the series terminates: exact up to rounding)."""
    nx, nu = B.shape
    M = np.zeros((nx + nu, nx + nu))
    M[:nx, :nx], M[:nx, nx:] = A * dt, B * dt
    E, T = np.eye(nx + nu), np.eye(nx + nu)
    for k in range(1, 24):
        T = T @ M / k
        if not T.any():
            break
        E = E + T
    return E[:nx, :nx], E[:nx, nx:]


def quadrotor_plants(seed: int, start: int, count: int):
    """Config 4 plants for global indices start .. start+count-1: mass and the three inertias scaled
    by U(1 - spread, 1 + spread) each (counter-based draws 0..3), ZOH at dt.  A does not depend on
    mass or inertia, so Ad and Phi = int_0^dt exp(A s) ds are those of the nominal model (the
    augmented series of zoh() with B = I) and Bd = Phi B(plant).  Returns Ad (count, 12, 12),
    Bd (count, 12, 4)."""
    q = QUAD
    u = uniforms(seed, start, count, 4)
    f = 1.0 + q["spread"] * (2.0 * u - 1.0)
    A, _ = quadrotor_continuous(q["mass"], *q["inertia"], q["g"])
    Ad0, Phi = zoh(A, np.eye(12), q["dt"])
    Bc = np.zeros((count, 12, 4))
    Bc[:, 8, 0] = 1.0 / (q["mass"] * f[:, 0])
    Bc[:, 9, 1] = 1.0 / (q["inertia"][0] * f[:, 1])
    Bc[:, 10, 2] = 1.0 / (q["inertia"][1] * f[:, 2])
    Bc[:, 11, 3] = 1.0 / (q["inertia"][2] * f[:, 3])
    Ad = np.broadcast_to(Ad0, (count, 12, 12)).copy()
    Bd = np.einsum("ij,bjk->bik", Phi, Bc)
    return Ad, Bd


def quadrotor_shared() -> dict:
    """The weights and constraint data shared by every config-4 plant (mpc_mimo.h names): Cd = I,
    Q, R, RD diagonal, K = 0 (no state term in the bounds), K0 = I (box on the applied input), w0."""
    q = QUAD
    return {"Cd": np.eye(12), "Q": np.diag(q["q_diag"]), "R": np.diag(q["r_diag"]), "RD": np.diag(q["rd_diag"]),
            "K": np.zeros((4, 12)), "K0": np.eye(4), "w0": np.array(q["w0"], dtype=np.float64)}


def quadrotor_states(seed: int, start: int, count: int):
    """Config 4 states X ~ N(0, diag(QUAD_X_STD^2)) and applied inputs U ~ U(-w0/2, w0/2)."""
    X = normals(seed, start, count, 12) * QUAD_X_STD
    U = (uniforms(seed ^ 0x5A5A, start, count, 4) - 0.5) * np.array(QUAD["w0"])
    return X, U


def flops_mimo_setup(N: int, nx: int, nu: int, ny: int, scaling: int = 10) -> float:
    """FLOPs mimo_setup_kernel performs per plant (structured condensing, mpcq_mimo.hip): the CS / Sx
    recurrences, Fx, Q CS, the prefix-sum H, Fu, Frs, P assembly, and `scaling` Ruiz passes over P
    (column norms twice, rescale once)."""
    n = N * nu
    rec = N * 2 * (ny * nu * nx + 2 * ny * nx * nx + nx * nu * nx + ny * nx * ny)
    fx = sum(d + 1 for d in range(N)) * 2 * nu * nx * ny
    qcs = N * 2 * ny * nu * ny
    h = sum(N - d for d in range(N)) * 2 * nu * nu * ny
    fu = sum(N - j for j in range(N)) * 2 * nu * nu * ny
    frs = sum(N - j for j in range(N)) * nu * ny
    ruiz = scaling * 3 * n * n
    return float(rec + fx + qcs + h + fu + frs + 4 * n * n + ruiz)


def flops_mimo_solve(n: int, nu: int, iters, factorisations, check: int = 25) -> np.ndarray:
    """FLOPs mimo_solve_kernel performs per QP: 2 n^3 per Gauss-Jordan inverse of the reduced KKT
    matrix (initial + one per adaptive-rho change), and per iteration the GEMV with M^-1 (2 n^2), the
    structured A^ / A^' products (block scans and K0 products, 2 x (2 n nu + n log2(64/nu)) each, plus
    A^'A^ x~ for the carried P^ x) and ~30 n of element-wise work; per check two more products and
    the norms (~20 n)."""
    it = np.asarray(iters, dtype=np.float64)
    sc = 2 * n * nu + n * np.log2(64 / nu)
    f_iter = 2 * n * n + 2 * sc + 30 * n
    f_check = 2 * sc + 20 * n
    return np.asarray(factorisations, dtype=np.float64) * 2 * n ** 3 + it * f_iter + np.floor(it / check) * f_check


def flops_mimo_dense(N: int, nx: int, nu: int, ny: int, iters, check: int = 25) -> np.ndarray:
    """Dense-equivalent count: dense condensing 2 (N nu)^2 (N ny) + Ruiz 10 x 3 (n^2 + nm)
    + one KKT LDL 2 n^2 m + n^3 / 3 + n^2, and iters x F_iter + checks x F_check with
    F_iter = 4nm + 2n^2 + 9m + 6n, F_check = 4nm + 2n^2 + 6m + 4n."""
    n, m = N * nu, 2 * N * nu
    it = np.asarray(iters, dtype=np.float64)
    setup = 2 * n * n * (N * ny) + 30 * (n * n + n * m) + 2 * n * n * m + n ** 3 / 3 + n * n
    return setup + it * (4 * n * m + 2 * n * n + 9 * m + 6 * n) + np.floor(it / check) * (4 * n * m + 2 * n * n + 6 * m + 4 * n)
