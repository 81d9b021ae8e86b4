"""Python mirror of the reference's ``ModelPredictiveControlAPI`` (include/ModelPredictiveControlAPI.h,
src/ModelPredictiveControlAPI.cpp), on top of the MI355X solver.

Same names, argument meaning and error behaviour as the reference where they exist:
``from_json`` shape rules (:418-489), the ``set*`` builders, ``controllerStep`` (:81-108) returning
False on a solver failure, public ``X``, ``U``, ``dt``, ``verbose``, ``solverFlag``, ``n_variables``,
``n_constraints``, ``cfg``.  The horizon is a constructor argument (the reference's compile-time
``mpcWindow = 15``, ModelPredictiveControlAPI.h:26).  Condensing runs on the device
(``mpcq_condense``); the QP solve runs in the batched ADMM kernel.  ``batch > 1`` runs that many
copies of the controller (one per plant state) in lock-step, which is the benchmark workload.
"""
from __future__ import annotations

import ctypes as C
import json
from pathlib import Path

import numpy as np

from . import _capi

MPC_WINDOW = 15  # reference default (ModelPredictiveControlAPI.h:26)
N_S = 4          # states (ModelPredictiveControlAPI.h:28)
S_ROWS = 10      # rows of S set to K (ModelPredictiveControlAPI.cpp:185)


class JsonTypeError(TypeError):
    """Stands for nlohmann::detail::type_error thrown by the reference's from_json."""


def from_json(obj, rows: int, cols: int) -> np.ndarray:
    """JSON value -> matrix with the reference's shape rules (ModelPredictiveControlAPI.cpp:418-489):
    a scalar, a row/column vector or a matrix; an empty array returns an uninitialised rows x cols
    matrix (zeros here); a size mismatch or ragged rows raises."""
    if isinstance(obj, list):
        if len(obj) == 0:
            return np.zeros((rows, cols))
        arr = obj
    elif isinstance(obj, (int, float)) and not isinstance(obj, bool):
        arr = [obj]
    else:
        raise JsonTypeError("expected a number or an array")
    if isinstance(arr[0], list):
        aoa = arr
    elif rows == 1:
        aoa = [arr]
    elif cols == 1:
        aoa = [[v] for v in arr]
    else:
        raise JsonTypeError("Expected a matrix, received a vector.")
    pr, pc = len(aoa), len(aoa[0])
    if (rows >= 0 and pr != rows) or (cols >= 0 and pc != cols):
        raise JsonTypeError(f"Expected matrix of size {rows}x{cols}, received matrix of size {pr}x{pc}.")
    out = np.zeros((pr, pc))
    for r in range(pr):
        if len(aoa[r]) != pc:
            raise JsonTypeError("Unconsistent matrix size: some rows have different number of columns.")
        for c in range(pc):
            v = aoa[r][c]
            if not isinstance(v, (int, float)) or isinstance(v, bool):
                raise JsonTypeError("matrix entries must be numbers")
            out[r, c] = float(v)
    return out


def condense(plants: dict, N: int, s_rows: int = S_ROWS, device: int = 0) -> dict:
    """Batched condensing on the device (mpcq_condense).  ``plants`` holds arrays with a leading
    plant axis: Ad (k,nx,nx), Bd (k,nx), Cd (k,nx), K (k,nx), Q/R/RD (k,)."""
    Ad = np.ascontiguousarray(plants["Ad"], dtype=np.float64)
    k, nx = Ad.shape[0], Ad.shape[1]
    ins = [Ad] + [np.ascontiguousarray(plants[key], dtype=np.float64).reshape(k, -1) for key in ("Bd", "Cd", "K")]
    ins += [np.ascontiguousarray(plants[key], dtype=np.float64).reshape(k) for key in ("Q", "R", "RD")]
    shapes = {"P": (k, N, N), "A": (k, 2 * N, N), "Fx": (k, N, nx), "Fu": (k, N), "Fr": (k, N, N),
              "Sbar": (k, 2 * N, nx), "Ku": (k, 2 * N), "W0": (k, 2 * N)}
    out = {key: np.zeros(s) for key, s in shapes.items()}
    dp = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))  # noqa: E731
    rc = _capi.lib().mpcq_condense(device, k, nx, N, s_rows, *[dp(a) for a in ins],
                                   *[dp(out[key]) for key in ("P", "A", "Fx", "Fu", "Fr", "Sbar", "Ku", "W0")])
    _capi.check(rc, "mpcq_condense")
    return out


class ModelPredictiveControlAPI:
    """ModelPredictiveControlAPI(verbose) of the reference, batched over ``batch`` plant states."""

    def __init__(self, verbose: bool = False, config: str | Path = "./config/MPC_API.json",
                 N: int = MPC_WINDOW, batch: int = 1, dtype: str = "f64", device: int = 0,
                 settings=None):
        from . import BatchSolver, default_settings  # late import (package init order)
        print("[MPC API]\tMPC API object created.")
        self.verbose = bool(verbose)
        self.solverFlag = True
        self.N, self.batch, self.device = int(N), int(batch), int(device)
        self.cfg = json.loads(Path(config).read_text())  # throws like json::parse on a bad file
        self.K = from_json(self.cfg["K"], 1, N_S)
        self.xref = float(self.cfg["xref"])
        self.X = np.zeros((self.batch, N_S))
        self.U = np.zeros(self.batch)
        self.t0 = 0.0
        self.dt = 0.0
        self.setSystemVars()
        self.setCosts()
        self._ops = condense({"Ad": self.Ad[None], "Bd": self.Bd.reshape(1, -1), "Cd": self.Cd.reshape(1, -1),
                              "K": self.K.reshape(1, -1), "Q": [self.Q[0, 0]], "R": [self.R[0, 0]],
                              "RD": [self.RD[0, 0]]}, self.N, device=self.device)
        for key in ("P", "A", "Fx", "Fu", "Fr", "Sbar", "Ku", "W0"):
            setattr(self, key, self._ops[key][0])
        self.H, self.Gbar = self.P, self.A
        self.updateRef(self.xref)
        self.setF()
        # lb = -DBL_MAX (:42); ub = W0 + Sbar X + Ku U (:43)
        self.lb = np.full(2 * self.N, -np.finfo(np.float64).max)
        self.ub = self.W0 + self.Sbar @ self.X[0] + self.Ku * self.U[0]
        print("[MPC API]\tAll QP matrices built successfully.")
        self.n_variables = self.N
        self.n_constraints = 2 * self.N
        self.solver = BatchSolver(self.n_variables, self.n_constraints, self.batch, 1, dtype, self.device,
                                  settings or default_settings(verbose=int(self.verbose)))
        try:
            self.solver.setup(self.H, self.f[0], self.Gbar, self.lb, self.ub)
            self.solver.mpc_set_operators(self.Fx, self.Fu, self.Fr, self.Sbar, self.Ku, self.W0)
        except _capi.MpcqError:
            self.solverFlag = False

    def setVerbosity(self, verbose: bool) -> None:
        self.verbose = bool(verbose)
        print(f"[MPC API]\tVerbosity set to {int(self.verbose)}")

    def setSystemVars(self) -> None:
        self.Ad = from_json(self.cfg["Ad"], N_S, N_S)
        self.Bd = from_json(self.cfg["Bd"], N_S, 1)
        self.Cd = from_json(self.cfg["Cd"], 1, N_S)
        self.Dd = from_json(self.cfg["Dd"], 1, 1)

    def setCosts(self) -> None:
        self.Q = from_json(self.cfg["Q"], 1, 1)
        self.R = from_json(self.cfg["R"], 1, 1)
        self.RD = from_json(self.cfg["RD"], 1, 1)

    def updateRef(self, pos_ref: float) -> None:
        self.ref = np.full(self.N, float(pos_ref))

    def setF(self) -> None:
        """q = Fx X + Fu U + Fr ref' for every copy (ModelPredictiveControlAPI.cpp:372-375)."""
        self.f = self.X @ self.Fx.T + self.U[:, None] * self.Fu + self.Fr @ self.ref

    def controllerStep(self) -> bool:
        """One receding-horizon step (ModelPredictiveControlAPI.cpp:81-108) for every copy: q, u,
        warm-started solve, U += x[0].  False when any copy's solve did not reach OSQP_SOLVED."""
        self.t0 += self.dt
        self.updateRef(self.xref)
        self.U = self.solver.mpc_step(self.X, self.U, self.xref)
        status, _, _ = self.solver.info()
        return bool(np.all(status == _capi.SOLVED))

    def getSolution(self) -> np.ndarray:
        return self.solver.solution()
