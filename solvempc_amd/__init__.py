"""solvempc_amd — MI355X-native batched condensed-MPC QP solver (drop-in for the QP solve path of
LukeSchmitt96/solveMPC).

Python mirror of the C ABI in ``include/mpcq.h`` (library ``solvempc_amd/libmpcq.so``, built for
gfx950).  Names follow the reference's solver interface as it is used in
src/ModelPredictiveControlAPI.cpp (osqp-eigen: ``updateGradient`` / ``updateUpperBound`` /
``solve`` / ``getSolution``; OSQP settings and status values).  There is no CPU path: importing works
anywhere the library exists, but creating a solver needs a gfx950 device and fails loudly otherwise.
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import numpy as np

from . import _capi
from ._capi import (  # noqa: F401
    MPCQ_F32, MPCQ_F64, MPCQ_F64_MIXED, MPCQ_MIX_R, SOLVED, SOLVED_INACCURATE, MAX_ITER_REACHED, PRIMAL_INFEASIBLE,
    PRIMAL_INFEASIBLE_INACCURATE, DUAL_INFEASIBLE, DUAL_INFEASIBLE_INACCURATE, NON_CVX, UNSOLVED,
    INVALID_BOUNDS, TYPE_CHANGED, MpcqError, Settings, lib, library_path,
)

__all__ = ["BatchSolver", "Settings", "default_settings", "lib", "library_path", "MpcqError"]


def default_settings(**over) -> Settings:
    """OSQP v0.6 defaults + warm start (ModelPredictiveControlAPI.cpp:51-52)."""
    s = Settings()
    lib().mpcq_default_settings(C.byref(s))
    for k, v in over.items():
        if not hasattr(s, k):
            raise AttributeError(f"unknown setting {k}")
        setattr(s, k, v)
    return s


def _c64(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.float64))


def _dp(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_double))


class BatchSolver:
    """A batch of independent QPs  min 1/2 x'Px + q'x  s.t. l <= Ax <= u  on one gfx950 device.

    ``n_plants == 1``: all QPs share P and A (the reference's controller replicated over many
    states).  ``n_plants == batch``: one (P, A) per QP.
    """

    def __init__(self, n: int, m: int, batch: int, n_plants: int = 1, dtype: str = "f64",
                 device: int = 0, settings: Settings | None = None):
        self.n, self.m, self.batch, self.n_plants = int(n), int(m), int(batch), int(n_plants)
        self.dtype = dtype
        self.settings = settings or default_settings()
        codes = {"f64": MPCQ_F64, "f32": MPCQ_F32, "mixed": MPCQ_F64_MIXED}
        if dtype not in codes:
            raise ValueError(f"dtype {dtype!r}: one of {sorted(codes)}")
        dims = _capi.Dims(self.n, self.m, self.batch, self.n_plants, codes[dtype], int(device))
        ctx = C.c_void_p()
        _capi.check(lib().mpcq_create(C.byref(dims), C.byref(self.settings), C.byref(ctx)), "mpcq_create")
        self._ctx = ctx
        self.nx = 0

    def close(self):
        ctx = getattr(self, "_ctx", None)
        if ctx:
            self._ctx = None
            try:
                lib().mpcq_destroy(ctx)
            except TypeError:  # interpreter shutdown: module globals already torn down
                pass

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # -- setup: setHessianMatrix / setGradient / setLinearConstraintsMatrix / set*Bound + initSolver
    def setup(self, P, q0, A, l0, u0) -> None:
        k = self.n_plants
        P = _c64(P).reshape(k, self.n, self.n)
        q0 = _c64(q0).reshape(k, self.n)
        A = _c64(A).reshape(k, self.m, self.n)
        l0 = _c64(l0).reshape(k, self.m)
        u0 = _c64(u0).reshape(k, self.m)
        _capi.check(lib().mpcq_setup(self._ctx, _dp(P), _dp(q0), _dp(A), _dp(l0), _dp(u0)), "mpcq_setup")

    # -- per-step updates (updateGradient :96, updateUpperBound :99)
    def update_lin_cost(self, q) -> None:
        q = _c64(q).reshape(self.batch, self.n)
        _capi.check(lib().mpcq_update_lin_cost(self._ctx, _dp(q)), "mpcq_update_lin_cost")

    update_gradient = update_lin_cost

    def update_upper_bound(self, u) -> None:
        u = _c64(u).reshape(self.batch, self.m)
        _capi.check(lib().mpcq_update_upper_bound(self._ctx, _dp(u)), "mpcq_update_upper_bound")

    def update_lower_bound(self, l) -> None:
        l = _c64(l).reshape(self.batch, self.m)
        _capi.check(lib().mpcq_update_lower_bound(self._ctx, _dp(l)), "mpcq_update_lower_bound")

    def update_bounds(self, l, u) -> None:
        l = _c64(l).reshape(self.batch, self.m)
        u = _c64(u).reshape(self.batch, self.m)
        _capi.check(lib().mpcq_update_bounds(self._ctx, _dp(l), _dp(u)), "mpcq_update_bounds")

    def warm_start(self, x, y) -> None:
        x = _c64(x).reshape(self.batch, self.n)
        y = _c64(y).reshape(self.batch, self.m)
        _capi.check(lib().mpcq_warm_start(self._ctx, _dp(x), _dp(y)), "mpcq_warm_start")

    def cold_start(self) -> None:
        _capi.check(lib().mpcq_cold_start(self._ctx), "mpcq_cold_start")

    def reset_state(self) -> None:
        """Back to the post-setup state (x = z = y = 0, rho = settings.rho) for the next solve."""
        _capi.check(lib().mpcq_reset(self._ctx), "mpcq_reset")

    # -- solve (:102) and results (:105)
    def solve(self, stream: int | None = None) -> None:
        _capi.check(lib().mpcq_solve(self._ctx, C.c_void_p(stream or 0)), "mpcq_solve")

    def solution(self) -> np.ndarray:
        x = np.empty((self.batch, self.n))
        _capi.check(lib().mpcq_get_solution(self._ctx, _dp(x)), "mpcq_get_solution")
        return x

    def dual(self) -> np.ndarray:
        y = np.empty((self.batch, self.m))
        _capi.check(lib().mpcq_get_dual(self._ctx, _dp(y)), "mpcq_get_dual")
        return y

    def info(self):
        st = np.empty(self.batch, dtype=np.int32)
        it = np.empty(self.batch, dtype=np.int32)
        rho = np.empty(self.batch)
        _capi.check(lib().mpcq_get_info(self._ctx, st.ctypes.data_as(C.POINTER(C.c_int)),
                                        it.ctypes.data_as(C.POINTER(C.c_int)), _dp(rho)), "mpcq_get_info")
        return st, it, rho

    def scaling(self):
        D, E, c = np.empty(self.n), np.empty(self.m), C.c_double()
        _capi.check(lib().mpcq_get_scaling(self._ctx, _dp(D), _dp(E), C.byref(c)), "mpcq_get_scaling")
        return D, E, c.value

    def path(self) -> tuple[str, bool]:
        """(kernel family of the next solve: "tile" / "wave" / "lane", paired tile loop)."""
        k, p = C.c_int(), C.c_int()
        _capi.check(lib().mpcq_get_path(self._ctx, C.byref(k), C.byref(p)), "mpcq_get_path")
        return ("tile", "wave", "lane")[k.value], bool(p.value)

    def stream_path(self) -> str:
        """How the last mpc_run_device call ran: "tile" / "wave" (one launch) or "graph" (per-step)."""
        k = C.c_int()
        _capi.check(lib().mpcq_get_stream_path(self._ctx, C.byref(k)), "mpcq_get_stream_path")
        return ("graph", "wave", "tile")[k.value]

    def order(self) -> tuple[bool, np.ndarray]:
        """(whether the last solve ran hardest-first, the QPs in the order phase 0 ran them: mpcq_get_order)."""
        o, lst = C.c_int(), np.zeros(self.batch, dtype=np.int32)
        _capi.check(lib().mpcq_get_order(self._ctx, C.byref(o), lst.ctypes.data_as(C.POINTER(C.c_int))),
                    "mpcq_get_order")
        return bool(o.value), lst

    def device_view(self) -> dict:
        v = _capi.DeviceView()
        _capi.check(lib().mpcq_device_view_get(self._ctx, C.byref(v)), "mpcq_device_view_get")
        return {k: int(getattr(v, k) or 0) for k, _ in _capi.DeviceView._fields_}

    # -- condensed-MPC front end (controllerStep, :81-108)
    def mpc_set_operators(self, Fx, Fu, Fr, Sbar, Ku, W0) -> None:
        k = self.n_plants
        Fx = _c64(Fx).reshape(k, self.n, -1)
        self.nx = Fx.shape[2]
        args = [Fx, _c64(Fu).reshape(k, self.n), _c64(Fr).reshape(k, self.n, self.n),
                _c64(Sbar).reshape(k, self.m, self.nx), _c64(Ku).reshape(k, self.m), _c64(W0).reshape(k, self.m)]
        _capi.check(lib().mpcq_mpc_set_operators(self._ctx, self.nx, *[_dp(a) for a in args]),
                    "mpcq_mpc_set_operators")

    def mpc_step(self, X, U, xref: float = 0.0) -> np.ndarray:
        """One receding-horizon step for every QP from host X (batch, nx), U (batch); returns new U."""
        X = _c64(X).reshape(self.batch, self.nx)
        U = _c64(U).reshape(self.batch).copy()
        _capi.check(lib().mpcq_mpc_step(self._ctx, _dp(X), _dp(U), float(xref)), "mpcq_mpc_step")
        return U

    # -- receding-horizon stream (BASELINE config 5): simulated plant + graph-captured control steps
    def mpc_set_plant(self, Ad, Bd) -> None:
        k = self.n_plants
        Ad = _c64(Ad).reshape(k, -1)
        nx = int(round(np.sqrt(Ad.shape[1])))
        Bd = _c64(Bd).reshape(k, nx)
        _capi.check(lib().mpcq_mpc_set_plant(self._ctx, nx, _dp(Ad), _dp(Bd)), "mpcq_mpc_set_plant")

    def mpc_simulate_device(self, X_ptr: int, U_ptr: int, seed: int, first_qp: int, step: int,
                            noise_std: float, stream: int | None = None) -> None:
        _capi.check(lib().mpcq_mpc_simulate_device(self._ctx, C.c_void_p(X_ptr), C.c_void_p(U_ptr), seed, first_qp,
                                                   step, float(noise_std), C.c_void_p(stream or 0)),
                    "mpcq_mpc_simulate_device")

    def mpc_run_device(self, X_ptr: int, U_ptr: int, xref: float, steps: int, seed: int, first_qp: int,
                       first_step: int, noise_std: float, stream: int) -> None:
        """``steps`` warm-started [controllerStep; plant update] rounds: one persistent launch on the
        one-QP-per-wave path (every wave runs its QP through all the steps), else replayed from a
        hipGraph."""
        _capi.check(lib().mpcq_mpc_run_device(self._ctx, C.c_void_p(X_ptr), C.c_void_p(U_ptr), float(xref),
                                              int(steps), seed, first_qp, first_step, float(noise_std),
                                              C.c_void_p(stream)), "mpcq_mpc_run_device")

    def stream_counters(self):
        """Per-QP (iterations, unsolved steps) accumulated over the last mpc_run_device call."""
        it = np.empty(self.batch, dtype=np.int32)
        un = np.empty(self.batch, dtype=np.int32)
        _capi.check(lib().mpcq_mpc_stream_counters(self._ctx, it.ctypes.data_as(C.POINTER(C.c_int)),
                                                   un.ctypes.data_as(C.POINTER(C.c_int))), "mpcq_mpc_stream_counters")
        return it, un

    def stream_iterations(self) -> np.ndarray:
        return self.stream_counters()[0]

    def stream_unsolved(self) -> int:
        return int(self.stream_counters()[1].sum())

    def mpc_setup_plants_device(self, nx: int, s_rows: int, Ad_ptr: int, Bd_ptr: int, Cd_ptr: int, K_ptr: int,
                                Q_ptr: int, R_ptr: int, RD_ptr: int, stream: int | None = None) -> None:
        """Condense and set up every plant on the device from device-resident plant data (fp64,
        plant-major; BASELINE config 3): the per-plant form of mpc.condense + setup +
        mpc_set_operators, with the ctor's X = U = 0 setup data."""
        ptrs = [C.c_void_p(p) for p in (Ad_ptr, Bd_ptr, Cd_ptr, K_ptr, Q_ptr, R_ptr, RD_ptr)]
        _capi.check(lib().mpcq_mpc_setup_plants_device(self._ctx, int(nx), int(s_rows), *ptrs,
                                                       C.c_void_p(stream or 0)), "mpcq_mpc_setup_plants_device")
        self.nx = int(nx)

    def mpc_plants_step_device(self, nx: int, s_rows: int, Ad_ptr: int, Bd_ptr: int, Cd_ptr: int, K_ptr: int,
                               Q_ptr: int, R_ptr: int, RD_ptr: int, X_ptr: int, U_ptr: int, xref: float = 0.0,
                               stream: int | None = None) -> None:
        """BASELINE config 3 in one pass: every plant's condensing + setup + one controllerStep (device
        pointers, plant-major fp64), operators kept on chip (the context keeps results only)."""
        ptrs = [C.c_void_p(p) for p in (Ad_ptr, Bd_ptr, Cd_ptr, K_ptr, Q_ptr, R_ptr, RD_ptr, X_ptr, U_ptr)]
        _capi.check(lib().mpcq_mpc_plants_step_device(self._ctx, int(nx), int(s_rows), *ptrs, float(xref),
                                                      C.c_void_p(stream or 0)), "mpcq_mpc_plants_step_device")

    # -- MIMO condensed MPC (BASELINE config 4; oracle/mpc_mimo.h formulation)
    def mimo_setup_plants_device(self, nx: int, nu: int, ny: int, s_rows: int, Ad_ptr: int, Bd_ptr: int, Cd_ptr: int,
                                 Q_ptr: int, R_ptr: int, RD_ptr: int, K_ptr: int, K0_ptr: int, w0_ptr: int,
                                 stream: int | None = None) -> None:
        """Condense and set up every plant on the device from device-resident, plant-major fp64 data
        (Ad nx*nx, Bd nx*nu, Cd ny*nx, Q ny*ny, R, RD nu*nu, K nu*nx, K0 nu*nu, w0 nu)."""
        ptrs = [C.c_void_p(p) for p in (Ad_ptr, Bd_ptr, Cd_ptr, Q_ptr, R_ptr, RD_ptr, K_ptr, K0_ptr, w0_ptr)]
        _capi.check(lib().mpcq_mimo_setup_plants_device(self._ctx, int(nx), int(nu), int(ny), int(s_rows), *ptrs,
                                                        C.c_void_p(stream or 0)), "mpcq_mimo_setup_plants_device")
        self.nx, self.nu = int(nx), int(nu)

    def mimo_step_device(self, X_ptr: int, U_ptr: int, yref_ptr: int = 0, stream: int | None = None) -> None:
        """One controllerStep for every QP on device-resident X (batch, nx), U (batch, nu); asynchronous."""
        _capi.check(lib().mpcq_mimo_step_device(self._ctx, C.c_void_p(X_ptr), C.c_void_p(U_ptr),
                                                C.c_void_p(yref_ptr or 0), C.c_void_p(stream or 0)),
                    "mpcq_mimo_step_device")

    def mpc_step_device(self, X_ptr: int, U_ptr: int, xref: float = 0.0, stream: int | None = None) -> None:
        """Same on device-resident fp64 buffers (e.g. torch tensors' data_ptr()); asynchronous."""
        _capi.check(lib().mpcq_mpc_step_device(self._ctx, C.c_void_p(X_ptr), C.c_void_p(U_ptr),
                                               float(xref), C.c_void_p(stream or 0)), "mpcq_mpc_step_device")


from .mpc import ModelPredictiveControlAPI, from_json  # noqa: E402,F401
