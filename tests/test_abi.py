"""CPU tests of the drop-in boundary: the C-ABI library loads, exports every symbol include/mpcq.h
declares, and fails loudly (no CPU fallback) when no gfx950 device is present."""
import re
import subprocess
from pathlib import Path

import numpy as np
import pytest

import solvempc_amd as sm
from solvempc_amd import _capi

ROOT = Path(__file__).resolve().parents[1]


def _declared():
    hdr = (ROOT / "include" / "mpcq.h").read_text()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    return set(re.findall(r"\b(mpcq_[a-z_0-9]+)\s*\(", hdr))


def test_header_matches_exports():
    assert _declared() == set(_capi.EXPORTS)


def test_library_exports_every_symbol():
    lib = sm.lib()
    missing = [s for s in _declared() if not hasattr(lib, s)]
    assert not missing


def test_default_settings_are_osqp_v06():
    s = sm.default_settings()
    assert (s.rho, s.sigma, s.alpha, s.eps_abs, s.eps_rel) == (0.1, 1e-6, 1.6, 1e-3, 1e-3)
    assert (s.max_iter, s.check_termination, s.scaling, s.adaptive_rho, s.warm_start) == (4000, 25, 10, 1, 1)
    assert s.adaptive_rho_tolerance == 5.0 and s.scaled_termination == 0


def _has_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.mark.skipif(_has_gpu(), reason="checks the no-device failure mode")
def test_no_device_fails_loudly():
    with pytest.raises(sm.MpcqError) as e:
        sm.BatchSolver(20, 40, 16)
    assert e.value.code == _capi.MPCQ_ERR_HIP


def test_argument_errors():
    with pytest.raises(sm.MpcqError) as e:
        sm.BatchSolver(20, 40, 16, n_plants=3)
    assert e.value.code == _capi.MPCQ_ERR_ARG
    with pytest.raises(AttributeError):
        sm.default_settings(not_a_setting=1)


@pytest.mark.skipif(_has_gpu(), reason="checks the no-device failure mode")
def test_cli_fails_without_device(tmp_path):
    exe = ROOT / "solvempc_amd" / "solvempc"
    assert exe.exists(), "build() produces the solver.cpp-compatible CLI"
    cfg = ROOT / "tests" / "golden" / "plant_mpc_api.json"
    r = subprocess.run([str(exe), "-c", str(cfg)], input="", capture_output=True, text=True, timeout=60)
    assert r.returncode != 0


def test_condense_from_json_shapes():
    from solvempc_amd import mpc
    np.testing.assert_array_equal(mpc.from_json([5.0], 1, 1), [[5.0]])        # RD given as [5.0]
    np.testing.assert_array_equal(mpc.from_json(2.0, 1, 1), [[2.0]])
    np.testing.assert_array_equal(mpc.from_json([1, 2, 3, 4], 4, 1), [[1], [2], [3], [4]])
    with pytest.raises(mpc.JsonTypeError):
        mpc.from_json([[1, 2], [3]], 2, 2)
    with pytest.raises(mpc.JsonTypeError):
        mpc.from_json([1, 2, 3], 4, 1)


def test_header_constants_match_the_mirror():
    """The precision constants of include/mpcq.h (MPCQ_F64 / F32 / F64_MIXED and the mixed path's fp64
    share MPCQ_MIX_R) are the ctypes mirror's: bench.py prices the mixed FLOP split with the latter."""
    hdr = (ROOT / "include" / "mpcq.h").read_text()
    for name in ("MPCQ_F64", "MPCQ_F32", "MPCQ_F64_MIXED", "MPCQ_MIX_R"):
        m = re.search(rf"#define {name} (\d+)", hdr)
        assert m and int(m.group(1)) == getattr(_capi, name), name


def test_flop_accounting_helpers():
    """workload's FLOP counts: the mixed split adds up to the total (per solve and over a stream whose solves
    stop on check iterations), and the fp64 per-plant kernel's one-GEMV count is below the two-product one
    by exactly the per-iteration and per-factorisation difference."""
    from solvempc_amd import workload as w
    it = np.array([25, 50, 75, 100, 125, 225, 13])
    f64, f32 = w.flops_split_mixed(20, 40, 4, it, 5, paired=True)
    assert np.allclose(f64 + f32, w.flops_per_qp(20, 40, 4, it, paired=True))
    assert np.all(f32[:6] == (it[:6] - (it[:6] // 25) * 5) * w._flop_terms(20, 40, 4, True)[0])
    tot = np.array([25 * 1000, 25 * 1003, 50 * 1000])
    g64, g32 = w.flops_split_mixed_total(20, 40, 4, tot, 1000, 5, paired=True)
    assert np.allclose(g64 + g32, w.flops_per_qp_total(20, 40, 4, tot, 1000, paired=True))
    iters, ref = np.array([97.0, 125.0]), np.array([0.0, 1.0])
    a = w.flops_plant_step(20, 4, iters, ref)
    b = w.flops_plant_step(20, 4, iters, ref, merged=True)
    N = 20
    assert np.allclose(a - b, iters * (2 * N * N - 5 * N) + (1 + ref) * 4 * N * N)
