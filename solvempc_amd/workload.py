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


def randomized_plants(plant: dict, seed: int, start: int, count: int, rel: float = 0.02, attempts: int = 64):
    """Config 3 plants for global indices start .. start+count-1: Ad = Ad0 o (1 + rel eps),
    Bd = Bd0 o (1 + rel eps), eps ~ N(0, 1) (Box-Muller on draws 32a .. 32a+19 of attempt a); a draw
    with spectral radius rho(Ad) >= 1 is rejected and redrawn (after `attempts` the nominal plant)."""
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
    paired: the tile kernel's paired loop (rows n + j of A = -rows j) performs B'w and B eta over
    m/2 rows, F_iter = 2nm + 2n^2 + 9m + 6n (the reduced count it actually performs; SURVEY §8d asks
    for it when the A structure is exploited); its check iterations keep the dense F_check."""
    it = np.asarray(iters, dtype=np.float64)
    f_iter = (2 if paired else 4) * n * m + 2 * n * n + 9 * m + 6 * n
    f_check = 4 * n * m + 2 * n * n + 6 * m + 4 * n
    f_front = 2 * n * (nx + 1 + n) + 2 * m * (nx + 1) + 2 * n * n
    return it * f_iter + np.floor(it / check) * f_check + f_front


def flops_plant_setup(n: int, m: int, N: int | None = None) -> float:
    """Algorithmic FLOPs of one plant's condensing + setup: F_condense (SISO)
    4N^3 + 10N^2 + 128N, Ruiz 10*3(n^2 + nm), F_setup 2n^2 m + n^3/3 + n^2 (one LDL of the KKT
    system; the eigen-basis setup does more work than this and is not credited for it)."""
    N = n if N is None else N
    return (4 * N ** 3 + 10 * N ** 2 + 128 * N) + 30 * (n * n + n * m) + (2 * n * n * m + n ** 3 / 3 + n * n)
