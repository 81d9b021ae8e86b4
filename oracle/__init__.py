"""oracle — TEST INFRASTRUCTURE ONLY.

ctypes binding of the plain-C CPU checker in this directory:

* ``mpc_condense.c`` restates the condensed-QP construction of LukeSchmitt96/solveMPC
  (src/ModelPredictiveControlAPI.cpp:111-375), pinned against the known-answer values of
  SURVEY.md Appendix B;
* ``mpc_mimo.c`` generalises that construction to n_u inputs / n_y outputs (BASELINE config 4; no
  reference counterpart — its SISO specialisation is ``mpc_condense.c``'s arithmetic);
* ``osqp_dense.c`` restates OSQP v0.6's ADMM (the un-vendored solver behind
  ModelPredictiveControlAPI.cpp:51-64,96-105) in dense fp64.  PARITY UNPINNED at that
  boundary (no OSQP build, no reference fixtures); certified by KKT optimality checks.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this package, and only as the checker / the timed CPU baseline.  The product
(``solvempc_amd``) never imports it.
"""
from __future__ import annotations

import ctypes as C
import json
import os
import subprocess
from pathlib import Path

import numpy as np

_HERE = Path(__file__).resolve().parent
_LIB = None

SOLVED, SOLVED_INACCURATE, MAX_ITER_REACHED = 1, 2, -2
PRIMAL_INFEASIBLE, DUAL_INFEASIBLE, NON_CVX, UNSOLVED = -3, -4, -7, -10


class Settings(C.Structure):
    _fields_ = [
        ("rho", C.c_double), ("sigma", C.c_double), ("alpha", C.c_double),
        ("eps_abs", C.c_double), ("eps_rel", C.c_double),
        ("eps_prim_inf", C.c_double), ("eps_dual_inf", C.c_double),
        ("adaptive_rho_tolerance", C.c_double), ("adaptive_rho_fraction", C.c_double),
        ("max_iter", C.c_int), ("check_termination", C.c_int), ("scaling", C.c_int),
        ("adaptive_rho", C.c_int), ("adaptive_rho_interval", C.c_int),
        ("warm_start", C.c_int), ("scaled_termination", C.c_int),
    ]


class Info(C.Structure):
    _fields_ = [
        ("iter", C.c_int), ("status", C.c_int), ("rho_updates", C.c_int),
        ("pri_res", C.c_double), ("dua_res", C.c_double),
        ("rho_estimate", C.c_double), ("rho", C.c_double),
        ("margin", C.c_double),  # smallest |ln(value / threshold)| of the solve's schedule decisions
    ]


class _Plant(C.Structure):
    _fields_ = [
        ("nx", C.c_int), ("N", C.c_int), ("s_rows", C.c_int),
        ("Ad", C.POINTER(C.c_double)), ("Bd", C.POINTER(C.c_double)),
        ("Cd", C.POINTER(C.c_double)), ("K", C.POINTER(C.c_double)),
        ("Q", C.c_double), ("R", C.c_double), ("RD", C.c_double),
    ]


class _MimoPlant(C.Structure):
    _fields_ = [("nx", C.c_int), ("nu", C.c_int), ("ny", C.c_int), ("N", C.c_int), ("s_rows", C.c_int)] + \
               [(k, C.POINTER(C.c_double)) for k in ("Ad", "Bd", "Cd", "Q", "R", "RD", "K", "K0", "w0")]


class _MimoOps(C.Structure):
    _fields_ = [(k, C.POINTER(C.c_double)) for k in ("P", "A", "Fx", "Fu", "Fr", "Sbar", "Ku", "W0", "Su")]


class _Ops(C.Structure):
    _fields_ = [(k, C.POINTER(C.c_double)) for k in
                ("P", "A", "Fx", "Fu", "Fr", "Sbar", "Ku", "W0", "Su", "Sx")]


def lib() -> C.CDLL:
    """Load (building on first use if needed) oracle/liboracle.so."""
    global _LIB
    if _LIB is not None:
        return _LIB
    so = _HERE / "liboracle.so"
    srcs = [_HERE / f for f in ("mpc_condense.c", "osqp_dense.c", "mpc_batch.c", "mpc_condense.h", "osqp_dense.h",
                                "mpc_batch.h", "mpc_mimo.c", "mpc_mimo.h")]
    if os.environ.get("ORACLE_LIB"):  # the ASan / UBSan build (make sanitize), libasan preloaded
        so = Path(os.environ["ORACLE_LIB"])
    elif not so.exists() or any(s.stat().st_mtime > so.stat().st_mtime for s in srcs if s.exists()):
        subprocess.run(["make", "-C", str(_HERE), "-s"], check=True)
    L = C.CDLL(str(so))
    dp = C.POINTER(C.c_double)
    ip = C.POINTER(C.c_int)
    L.ora_default_settings.argtypes = [C.POINTER(Settings)]
    L.ora_setup.restype = C.c_void_p
    L.ora_setup.argtypes = [C.c_int, C.c_int, dp, dp, dp, dp, dp, C.POINTER(Settings)]
    L.ora_cleanup.argtypes = [C.c_void_p]
    L.ora_update_lin_cost.argtypes = [C.c_void_p, dp]
    L.ora_update_upper_bound.argtypes = [C.c_void_p, dp]
    L.ora_update_lower_bound.argtypes = [C.c_void_p, dp]
    L.ora_update_bounds.argtypes = [C.c_void_p, dp, dp]
    L.ora_warm_start.argtypes = [C.c_void_p, dp, dp]
    L.ora_cold_start.argtypes = [C.c_void_p]
    L.ora_solve.argtypes = [C.c_void_p]
    L.ora_solution_x.restype = dp
    L.ora_solution_x.argtypes = [C.c_void_p]
    L.ora_solution_y.restype = dp
    L.ora_solution_y.argtypes = [C.c_void_p]
    L.ora_get_info.argtypes = [C.c_void_p, C.POINTER(Info)]
    L.ora_get_scaling.argtypes = [C.c_void_p, dp, dp, dp]
    L.ora_get_iterates.argtypes = [C.c_void_p, dp, dp, dp]
    L.ora_batch_solve.restype = C.c_int
    L.ora_batch_solve.argtypes = [C.c_int, C.c_int, dp, dp, dp, dp, dp, C.POINTER(Settings),
                                  C.c_int, dp, dp, dp, ip, ip, dp, C.c_int, dp]
    L.ora_condense.argtypes = [C.POINTER(_Plant), C.POINTER(_Ops)]
    L.ora_condense.restype = C.c_int
    L.ora_matpow.argtypes = [C.c_int, dp, C.c_int, dp]
    L.ora_plants_step.restype = C.c_int
    L.ora_plants_step.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, dp, dp, dp, dp, C.c_double, C.c_double,
                                  C.c_double, dp, dp, C.c_double, C.POINTER(Settings), dp, ip, ip, C.c_int, dp, dp]
    L.ora_stream_run.restype = C.c_int
    L.ora_stream_run.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, dp, dp, dp, dp, C.c_double, C.c_double,
                                 C.c_double, dp, dp, C.c_double, C.POINTER(Settings), C.c_int, C.c_ulonglong,
                                 C.c_longlong, C.c_longlong, C.c_double, ip, ip, C.c_int]
    L.ora_condense_mimo.restype = C.c_int
    L.ora_condense_mimo.argtypes = [C.POINTER(_MimoPlant), C.POINTER(_MimoOps)]
    L.ora_mimo_plants_step.restype = C.c_int
    L.ora_mimo_plants_step.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, dp, dp, dp, dp, dp, dp,
                                       dp, dp, dp, dp, dp, dp, C.POINTER(Settings), dp, dp, ip, ip, C.c_int, dp]
    _LIB = L
    return L


def _dp(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def _ip(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_int))


def _c64(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.float64))


def default_settings(**over) -> Settings:
    s = Settings()
    lib().ora_default_settings(C.byref(s))
    for k, v in over.items():
        setattr(s, k, v)
    return s


# ----------------------------------------------------------------------------- condensing
def load_plant(path: str | os.PathLike) -> dict:
    """Read the plant/weights from an MPC_API.json-shaped file (numbers only)."""
    cfg = json.loads(Path(path).read_text())
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


def condense(plant: dict, N: int, s_rows: int = 10) -> dict:
    """Condensed operators (ModelPredictiveControlAPI.cpp:180-368) as fp64 numpy arrays."""
    nx = plant["Ad"].shape[0]
    keep = {k: _c64(plant[k]) for k in ("Ad", "Bd", "Cd", "K")}
    pl = _Plant(nx, N, s_rows, _dp(keep["Ad"]), _dp(keep["Bd"]), _dp(keep["Cd"]), _dp(keep["K"]),
                plant["Q"], plant["R"], plant["RD"])
    shapes = {"P": (N, N), "A": (2 * N, N), "Fx": (N, nx), "Fu": (N,), "Fr": (N, N),
              "Sbar": (2 * N, nx), "Ku": (2 * N,), "W0": (2 * N,), "Su": (N, N), "Sx": (N, nx)}
    out = {k: np.zeros(s, dtype=np.float64) for k, s in shapes.items()}
    ops = _Ops(*[_dp(out[k]) for k in ("P", "A", "Fx", "Fu", "Fr", "Sbar", "Ku", "W0", "Su", "Sx")])
    if lib().ora_condense(C.byref(pl), C.byref(ops)) != 0:
        raise ValueError("condense failed")
    return out


def gradient(ops: dict, X, U, xref: float = 0.0) -> np.ndarray:
    """q = Fx X + Fu U + Fr ref' (setF, ModelPredictiveControlAPI.cpp:372-375).  Batched in X."""
    X = np.asarray(X, dtype=np.float64)
    U = np.asarray(U, dtype=np.float64)
    ref = np.full(ops["Fr"].shape[1], xref)
    return X @ ops["Fx"].T + U[..., None] * ops["Fu"] + ops["Fr"] @ ref


def upper_bound(ops: dict, X, U) -> np.ndarray:
    """u = W0 + Sbar X + Ku U (ModelPredictiveControlAPI.cpp:43,99).  Batched in X."""
    X = np.asarray(X, dtype=np.float64)
    U = np.asarray(U, dtype=np.float64)
    return ops["W0"] + X @ ops["Sbar"].T + U[..., None] * ops["Ku"]


MIMO_KEYS = ("Ad", "Bd", "Cd", "Q", "R", "RD", "K", "K0", "w0")


def mimo_dims(plant: dict) -> tuple[int, int, int]:
    Bd = np.asarray(plant["Bd"])
    return Bd.shape[0], Bd.shape[1], np.asarray(plant["Cd"]).shape[0]


def condense_mimo(plant: dict, N: int, s_rows: int | None = None) -> dict:
    """MIMO condensed operators (mpc_mimo.h): plant dict with Ad (nx,nx), Bd (nx,nu), Cd (ny,nx),
    Q (ny,ny), R, RD (nu,nu), K (nu,nx), K0 (nu,nu), w0 (nu)."""
    nx, nu, ny = mimo_dims(plant)
    keep = {k: _c64(plant[k]) for k in MIMO_KEYS}
    pl = _MimoPlant(nx, nu, ny, N, N if s_rows is None else s_rows, *[_dp(keep[k]) for k in MIMO_KEYS])
    n, m = N * nu, 2 * N * nu
    shapes = {"P": (n, n), "A": (m, n), "Fx": (n, nx), "Fu": (n, nu), "Fr": (n, N * ny), "Sbar": (m, nx),
              "Ku": (m, nu), "W0": (m,), "Su": (N * ny, n)}
    out = {k: np.zeros(sh, dtype=np.float64) for k, sh in shapes.items()}
    ops = _MimoOps(*[_dp(out[k]) for k in ("P", "A", "Fx", "Fu", "Fr", "Sbar", "Ku", "W0", "Su")])
    if lib().ora_condense_mimo(C.byref(pl), C.byref(ops)) != 0:
        raise ValueError("condense_mimo failed")
    return out


def mimo_gradient(ops: dict, X, U, yref=None) -> np.ndarray:
    """q = Fx X + Fu U + Fr (1_N (x) yref).  Batched in X, U."""
    X, U = np.asarray(X, dtype=np.float64), np.asarray(U, dtype=np.float64)
    ny_tot = ops["Fr"].shape[1]
    ref = np.zeros(ny_tot) if yref is None else np.tile(np.asarray(yref, dtype=np.float64), ny_tot // len(yref))
    return X @ ops["Fx"].T + U @ ops["Fu"].T + ops["Fr"] @ ref


def mimo_upper_bound(ops: dict, X, U) -> np.ndarray:
    X, U = np.asarray(X, dtype=np.float64), np.asarray(U, dtype=np.float64)
    return ops["W0"] + X @ ops["Sbar"].T + U @ ops["Ku"].T


def mimo_plants_step(shared: dict, Ad, Bd, X, U, N: int, yref=None, settings: Settings | None = None,
                     nthreads: int = 0, s_rows: int | None = None, margins: bool = False):
    """Per-plant MIMO batch (config 4): condense + setup + one controllerStep per plant.
    Returns (U_new (k, nu), x (k, n), status, iters) and, with ``margins``, each QP's decision
    margin (Info.margin)."""
    Ad, Bd, X, U = _c64(Ad), _c64(Bd), _c64(X), _c64(U)
    k, nx, nu = Bd.shape
    ny = np.asarray(shared["Cd"]).shape[0]
    sh = {key: _c64(shared[key]) for key in ("Cd", "Q", "R", "RD", "K", "K0", "w0")}
    yr = _c64(np.zeros(ny) if yref is None else yref)
    s = settings or default_settings()
    n = N * nu
    U_out = np.zeros((k, nu))
    x_out = np.zeros((k, n))
    st = np.zeros(k, dtype=np.int32)
    it = np.zeros(k, dtype=np.int32)
    mg = np.zeros(k)
    lib().ora_mimo_plants_step(k, nx, nu, ny, N, N if s_rows is None else s_rows, _dp(Ad), _dp(Bd), _dp(sh["Cd"]),
                               _dp(sh["Q"]), _dp(sh["R"]), _dp(sh["RD"]), _dp(sh["K"]), _dp(sh["K0"]), _dp(sh["w0"]),
                               _dp(X), _dp(U), _dp(yr), C.byref(s), _dp(U_out), _dp(x_out), _ip(st), _ip(it), nthreads,
                               _dp(mg))
    return (U_out, x_out, st, it, mg) if margins else (U_out, x_out, st, it)


# ----------------------------------------------------------------------------- OSQP restatement
class Solver:
    """Single-QP OSQP-0.6 restatement (osqp-eigen call surface as used by the reference)."""

    def __init__(self, P, q, A, l, u, settings: Settings | None = None):
        self.P, self.q, self.A = _c64(P), _c64(q), _c64(A)
        self.l, self.u = _c64(l), _c64(u)
        self.n, self.m = self.P.shape[0], self.A.shape[0]
        self.settings = settings or default_settings()
        self._w = lib().ora_setup(self.n, self.m, _dp(self.P), _dp(self.q), _dp(self.A),
                                  _dp(self.l), _dp(self.u), C.byref(self.settings))
        if not self._w:
            raise ValueError("ora_setup rejected the problem data")

    def __del__(self):
        w = getattr(self, "_w", None)
        if w:
            lib().ora_cleanup(w)
            self._w = None

    def update_gradient(self, q) -> bool:
        q = _c64(q)
        return lib().ora_update_lin_cost(self._w, _dp(q)) == 0

    def update_upper_bound(self, u) -> bool:
        u = _c64(u)
        return lib().ora_update_upper_bound(self._w, _dp(u)) == 0

    def update_lower_bound(self, l) -> bool:
        l = _c64(l)
        return lib().ora_update_lower_bound(self._w, _dp(l)) == 0

    def update_bounds(self, l, u) -> bool:
        l, u = _c64(l), _c64(u)
        return lib().ora_update_bounds(self._w, _dp(l), _dp(u)) == 0

    def warm_start(self, x, y):
        x, y = _c64(x), _c64(y)
        lib().ora_warm_start(self._w, _dp(x), _dp(y))

    def cold_start(self):
        lib().ora_cold_start(self._w)

    def solve(self) -> int:
        lib().ora_solve(self._w)
        return self.info().status

    def x(self) -> np.ndarray:
        return np.ctypeslib.as_array(lib().ora_solution_x(self._w), shape=(self.n,)).copy()

    def y(self) -> np.ndarray:
        return np.ctypeslib.as_array(lib().ora_solution_y(self._w), shape=(self.m,)).copy()

    def info(self) -> Info:
        i = Info()
        lib().ora_get_info(self._w, C.byref(i))
        return i

    def scaling(self):
        D, E, c = np.zeros(self.n), np.zeros(self.m), C.c_double()
        lib().ora_get_scaling(self._w, _dp(D), _dp(E), C.byref(c))
        return D, E, c.value

    def iterates(self):
        x, z, y = np.zeros(self.n), np.zeros(self.m), np.zeros(self.m)
        lib().ora_get_iterates(self._w, _dp(x), _dp(z), _dp(y))
        return x, z, y


def batch_solve(P, A, q0, l, u0, q, u, settings: Settings | None = None, nthreads: int = 0,
                margins: bool = False):
    """Shared-template batch: setup(P,q0,A,l,u0) then per QP update q[b], u[b] and solve.
    Returns (x, status, iter, rho) and, with ``margins``, each QP's decision margin (Info.margin)."""
    P, A, q0, l, u0 = map(_c64, (P, A, q0, l, u0))
    q, u = _c64(q), _c64(u)
    n, m, B = P.shape[0], A.shape[0], q.shape[0]
    s = settings or default_settings()
    x = np.zeros((B, n))
    st = np.zeros(B, dtype=np.int32)
    it = np.zeros(B, dtype=np.int32)
    rho = np.zeros(B)
    mg = np.zeros(B)
    rc = lib().ora_batch_solve(n, m, _dp(P), _dp(A), _dp(q0), _dp(l), _dp(u0), C.byref(s), B,
                               _dp(q), _dp(u), _dp(x), _ip(st), _ip(it), _dp(rho), nthreads, _dp(mg))
    if rc < 0:
        raise ValueError("ora_batch_solve: setup rejected the data")
    return (x, st, it, rho, mg) if margins else (x, st, it, rho)


def plants_step(plant: dict, Ad, Bd, X, U, N: int, s_rows: int = 10, xref: float = 0.0,
                settings: Settings | None = None, nthreads: int = 0, full: bool = False):
    """Per-plant batch (config 3): for plant p with its own Ad[p], Bd[p] (Cd, K, Q, R, RD shared),
    the reference constructor + one controllerStep from (X[p], U[p]).  Returns (U_new, status, iter),
    and with ``full`` also the solutions x (k, N) and the decision margins (Info.margin)."""
    Ad, Bd, X, U = _c64(Ad), _c64(Bd), _c64(X), _c64(U)
    k, nx = Ad.shape[0], Ad.shape[1]
    Cd, K = _c64(plant["Cd"]), _c64(plant["K"])
    s = settings or default_settings()
    U_out = np.zeros(k)
    st = np.zeros(k, dtype=np.int32)
    it = np.zeros(k, dtype=np.int32)
    x = np.zeros((k, N))
    mg = np.zeros(k)
    lib().ora_plants_step(k, nx, N, s_rows, _dp(Ad), _dp(Bd), _dp(Cd), _dp(K), plant["Q"], plant["R"],
                          plant["RD"], _dp(X), _dp(U), float(xref), C.byref(s), _dp(U_out), _ip(st), _ip(it),
                          nthreads, _dp(x), _dp(mg))
    return (U_out, st, it, x, mg) if full else (U_out, st, it)


def kkt_residuals(P, q, A, l, u, x, y) -> dict:
    """Unscaled KKT residuals of min 1/2 x'Px + q'x s.t. l <= Ax <= u (independent of OSQP)."""
    P, A = np.asarray(P), np.asarray(A)
    Pu = np.triu(P)
    Pf = Pu + np.triu(P, 1).T
    Ax = A @ x
    stat = Pf @ x + q + A.T @ y
    prim = np.maximum(Ax - u, 0) + np.maximum(l - Ax, 0)
    yp, ym = np.maximum(y, 0), np.minimum(y, 0)
    dual_sign = np.where(u > 1e20, np.abs(yp), 0) + np.where(l < -1e20, np.abs(ym), 0)
    finite_u = np.where(u < 1e20, u, 0.0)
    finite_l = np.where(l > -1e20, l, 0.0)
    compl = np.abs(yp * (finite_u - Ax) * (u < 1e20)) + np.abs(ym * (finite_l - Ax) * (l > -1e20))
    return {
        "stationarity": float(np.abs(stat).max(initial=0.0)),
        "primal": float(prim.max(initial=0.0)),
        "dual_sign": float(dual_sign.max(initial=0.0)),
        "complementarity": float(compl.max(initial=0.0)),
    }


def stream_run(plant: dict, X, U, N: int, steps: int, seed: int, first_qp: int = 0, first_step: int = 0,
               noise_std: float = 1e-2, s_rows: int = 10, xref: float = 0.0, settings: Settings | None = None,
               nthreads: int = 0):
    """Config 5 on the CPU (oracle/mpc_batch.c ora_stream_run): every plant a copy of `plant` with its own
    warm-started solver, `steps` [controllerStep; plant update] rounds on the device's noise stream.
    Returns (X, U after the steps, per-plant iterations summed over the steps, unsolved steps)."""
    X, U = _c64(X).copy(), _c64(U).copy()
    k, nx = X.shape
    if not (1 <= N <= 64 and 1 <= nx <= 8):
        raise ValueError(f"stream_run: 1 <= N <= 64 and 1 <= nx <= 8 (got N={N}, nx={nx})")
    s = settings or default_settings()
    it = np.zeros(k, dtype=np.int32)
    un = np.zeros(k, dtype=np.int32)
    Ad, Bd, Cd, K = (_c64(plant[key]) for key in ("Ad", "Bd", "Cd", "K"))
    rc = lib().ora_stream_run(k, nx, N, s_rows, _dp(Ad), _dp(Bd), _dp(Cd), _dp(K), plant["Q"], plant["R"],
                              plant["RD"], _dp(X), _dp(U), xref, C.byref(s), steps, seed, first_qp, first_step,
                              noise_std, _ip(it), _ip(un), nthreads)
    if rc < 0:
        raise ValueError("ora_stream_run: setup rejected the plant")
    return X, U, it, un
