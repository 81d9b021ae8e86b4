"""ctypes declarations of include/mpcq.h (kept 1:1 with the header)."""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

MPCQ_OK, MPCQ_ERR_ARG, MPCQ_ERR_HIP, MPCQ_ERR_SETUP, MPCQ_ERR_ORDER, MPCQ_ERR_BOUNDS = 0, -1, -2, -3, -4, -5
SOLVED, SOLVED_INACCURATE, PRIMAL_INFEASIBLE_INACCURATE, DUAL_INFEASIBLE_INACCURATE = 1, 2, 3, 4
MAX_ITER_REACHED, PRIMAL_INFEASIBLE, DUAL_INFEASIBLE, NON_CVX, UNSOLVED = -2, -3, -4, -7, -10
INVALID_BOUNDS, TYPE_CHANGED = -20, -21
MPCQ_F64, MPCQ_F32, MPCQ_F64_MIXED = 0, 1, 2
MPCQ_MIX_R = 5  # include/mpcq.h: fp64 iterations per check interval of MPCQ_F64_MIXED

# Every symbol include/mpcq.h declares (tests check the library exports all of them).
EXPORTS = (
    "mpcq_default_settings", "mpcq_create", "mpcq_destroy", "mpcq_setup", "mpcq_update_lin_cost",
    "mpcq_update_upper_bound", "mpcq_update_lower_bound", "mpcq_update_bounds", "mpcq_warm_start",
    "mpcq_cold_start", "mpcq_reset", "mpcq_solve", "mpcq_get_solution", "mpcq_get_dual", "mpcq_get_info",
    "mpcq_get_scaling", "mpcq_device_view_get", "mpcq_mpc_set_operators", "mpcq_mpc_step_device",
    "mpcq_mpc_step", "mpcq_mpc_set_plant", "mpcq_mpc_simulate_device", "mpcq_mpc_run_device",
    "mpcq_condense", "mpcq_mpc_setup_plants_device", "mpcq_last_error", "mpcq_get_path",
    "mpcq_mimo_setup_plants_device", "mpcq_mimo_step_device", "mpcq_mpc_stream_counters",
    "mpcq_mpc_plants_step_device", "mpcq_get_stream_path", "mpcq_get_order",
)


class MpcqError(RuntimeError):
    def __init__(self, code: int, where: str, msg: str):
        super().__init__(f"{where} failed ({code}): {msg}")
        self.code = code


class Settings(C.Structure):
    _fields_ = [
        ("rho", C.c_double), ("sigma", C.c_double), ("alpha", C.c_double),
        ("eps_abs", C.c_double), ("eps_rel", C.c_double),
        ("eps_prim_inf", C.c_double), ("eps_dual_inf", C.c_double),
        ("adaptive_rho_tolerance", C.c_double), ("adaptive_rho_fraction", C.c_double),
        ("max_iter", C.c_int), ("check_termination", C.c_int), ("scaling", C.c_int),
        ("adaptive_rho", C.c_int), ("adaptive_rho_interval", C.c_int),
        ("warm_start", C.c_int), ("scaled_termination", C.c_int), ("verbose", C.c_int),
    ]


class Dims(C.Structure):
    _fields_ = [("n", C.c_int), ("m", C.c_int), ("batch", C.c_int), ("n_plants", C.c_int),
                ("dtype", C.c_int), ("device", C.c_int)]


class DeviceView(C.Structure):
    _fields_ = [("q", C.c_void_p), ("u", C.c_void_p), ("l", C.c_void_p), ("x", C.c_void_p),
                ("y", C.c_void_p), ("status", C.c_void_p), ("iter", C.c_void_p), ("rho", C.c_void_p)]


_LIB = None


def library_path() -> Path:
    return Path(os.environ.get("MPCQ_LIBRARY", Path(__file__).resolve().parent / "libmpcq.so"))


def lib() -> C.CDLL:
    """Load libmpcq.so.  Raises ImportError (never falls back) when it has not been built."""
    global _LIB
    if _LIB is not None:
        return _LIB
    path = library_path()
    if not path.exists():
        raise ImportError(f"{path} not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
    L = C.CDLL(str(path))
    dp, ip, vp = C.POINTER(C.c_double), C.POINTER(C.c_int), C.c_void_p
    sig = {
        "mpcq_default_settings": (None, [C.POINTER(Settings)]),
        "mpcq_create": (C.c_int, [C.POINTER(Dims), C.POINTER(Settings), C.POINTER(C.c_void_p)]),
        "mpcq_destroy": (C.c_int, [vp]),
        "mpcq_setup": (C.c_int, [vp, dp, dp, dp, dp, dp]),
        "mpcq_update_lin_cost": (C.c_int, [vp, dp]),
        "mpcq_update_upper_bound": (C.c_int, [vp, dp]),
        "mpcq_update_lower_bound": (C.c_int, [vp, dp]),
        "mpcq_update_bounds": (C.c_int, [vp, dp, dp]),
        "mpcq_warm_start": (C.c_int, [vp, dp, dp]),
        "mpcq_cold_start": (C.c_int, [vp]),
        "mpcq_reset": (C.c_int, [vp]),
        "mpcq_solve": (C.c_int, [vp, vp]),
        "mpcq_get_solution": (C.c_int, [vp, dp]),
        "mpcq_get_dual": (C.c_int, [vp, dp]),
        "mpcq_get_info": (C.c_int, [vp, ip, ip, dp]),
        "mpcq_get_scaling": (C.c_int, [vp, dp, dp, dp]),
        "mpcq_mimo_setup_plants_device": (C.c_int, [vp, C.c_int, C.c_int, C.c_int, C.c_int] + [vp] * 9 + [vp]),
        "mpcq_mimo_step_device": (C.c_int, [vp, vp, vp, vp, vp]),
        "mpcq_get_path": (C.c_int, [vp, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
        "mpcq_get_stream_path": (C.c_int, [vp, C.POINTER(C.c_int)]),
        "mpcq_get_order": (C.c_int, [vp, C.POINTER(C.c_int), ip]),
        "mpcq_device_view_get": (C.c_int, [vp, C.POINTER(DeviceView)]),
        "mpcq_mpc_set_operators": (C.c_int, [vp, C.c_int, dp, dp, dp, dp, dp, dp]),
        "mpcq_mpc_step_device": (C.c_int, [vp, vp, vp, C.c_double, vp]),
        "mpcq_mpc_step": (C.c_int, [vp, dp, dp, C.c_double]),
        "mpcq_mpc_set_plant": (C.c_int, [vp, C.c_int, dp, dp]),
        "mpcq_mpc_simulate_device": (C.c_int, [vp, vp, vp, C.c_ulonglong, C.c_longlong, C.c_longlong, C.c_double, vp]),
        "mpcq_mpc_run_device": (C.c_int, [vp, vp, vp, C.c_double, C.c_int, C.c_ulonglong, C.c_longlong,
                                          C.c_longlong, C.c_double, vp]),
        "mpcq_mpc_stream_counters": (C.c_int, [vp, ip, ip]),
        "mpcq_mpc_plants_step_device": (C.c_int, [vp, C.c_int, C.c_int] + [vp] * 9 + [C.c_double, vp]),
        "mpcq_condense": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int] + [dp] * 15),
        "mpcq_mpc_setup_plants_device": (C.c_int, [vp, C.c_int, C.c_int] + [vp] * 7 + [vp]),
        "mpcq_last_error": (C.c_char_p, []),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _LIB = L
    return L


def check(rc: int, where: str) -> None:
    if rc != MPCQ_OK:
        msg = lib().mpcq_last_error().decode(errors="replace")
        raise MpcqError(rc, where, msg)
