"""BASELINE config 4 (quad-rotor, n_x 12, n_u 4, N 30): the MIMO condensed-MPC path on the device
(mpcq_mimo_setup_plants_device + mpcq_mimo_step_device) against the CPU oracle (oracle/mpc_mimo.c:
condensing + OSQP-0.6 restatement), same plants and states.

The reference is SISO only, so the MIMO formulation is pinned two ways: its SISO specialisation is
bit-identical to the reference-pinned SISO condensing (test_oracle.py), and here the device path
run at n_u = 1 reproduces the reference controller's controllerStep.  Bar (fp64 throughout), on
EVERY QP: the oracle's status, and its iteration count with |x - x_oracle| <= 1e-7 max(1, |x|) and
the applied U to 1e-7.  Exception, counted and bounded: the device inverts the reduced KKT matrix
where the oracle factors the full KKT system (rounding ~1e-12 relative), so a QP whose schedule
decision the oracle itself takes within TIE_MARGIN of its threshold (|ln(residual / tolerance)|,
oracle Info.margin) may take the other branch; such a QP must still carry the oracle's status
(a SOLVED answer one check earlier or later, terminated by the device's own fp64 test).
"""
import numpy as np
import pytest

import oracle
import solvempc_amd as sm
from solvempc_amd import workload

pytestmark = pytest.mark.gpu
TIE_MARGIN = 1e-6


def _dev(a):
    import torch

    return torch.as_tensor(np.ascontiguousarray(a, dtype=np.float64), device="cuda:0")


def _run_device(shared, Ad, Bd, X, U, N, s_rows=None, yref=None, steps=1, settings=None):
    """Device path for a batch of plants; returns (U after each step, x, status, iters) of the last step."""
    import torch

    B, nx, nu = Bd.shape
    ny = np.asarray(shared["Cd"]).shape[0]
    keep = [_dev(Ad), _dev(Bd)] + [_dev(np.broadcast_to(np.asarray(shared[k], dtype=np.float64),
                                                        (B,) + np.asarray(shared[k]).shape).copy())
                                   for k in ("Cd", "Q", "R", "RD", "K", "K0", "w0")]
    s = sm.BatchSolver(N * nu, 2 * N * nu, B, n_plants=B, dtype="f64", settings=settings)
    stream = torch.cuda.current_stream().cuda_stream
    s.mimo_setup_plants_device(nx, nu, ny, N if s_rows is None else s_rows, *[k.data_ptr() for k in keep],
                               stream=stream)
    Xd, Ud = _dev(X), _dev(U)
    yd = _dev(yref) if yref is not None else None
    Us = []
    for _ in range(steps):
        s.mimo_step_device(Xd.data_ptr(), Ud.data_ptr(), yd.data_ptr() if yd is not None else 0, stream)
        torch.cuda.synchronize()
        Us.append(Ud.cpu().numpy().copy())
    st, it, _ = s.info()
    return Us, s.solution(), st, it


TIE_X_REL = 5e-2  # a tie's solution against the oracle's (as for config 3's fp32 ties, test_plants_step.py)


def _check(x, st, it, U1, x_ref, st_ref, it_ref, U_ref, margin, tol=1e-7):
    assert np.array_equal(st, st_ref), (st, st_ref)
    same = it == it_ref
    assert np.all(same | (margin < TIE_MARGIN)), (np.flatnonzero(~same), it[~same], it_ref[~same], margin[~same])
    if not same.all():
        print(f"{int((~same).sum())} of {len(same)} QPs took a tie's other branch (margins {margin[~same]})")
    rel = np.abs(x[same] - x_ref[same]).max(axis=1) / np.maximum(1.0, np.abs(x_ref[same]).max(axis=1))
    assert rel.max() < tol, rel.max()
    assert np.abs(U1[same] - U_ref[same]).max() < tol
    if not same.all():  # a tie stops one check earlier or later: both iterates met eps 1e-3, so they agree loosely
        rt = np.abs(x[~same] - x_ref[~same]).max(axis=1) / np.maximum(1.0, np.abs(x_ref[~same]).max(axis=1))
        assert rt.max() < TIE_X_REL, rt.max()


def test_quadrotor_step_matches_oracle():
    N, B = 30, 24
    Ad, Bd = workload.quadrotor_plants(3, 0, B)
    sh = workload.quadrotor_shared()
    X, U = workload.quadrotor_states(3, 0, B)
    Us, x, st, it = _run_device(sh, Ad, Bd, X, U, N)
    U_ref, x_ref, st_ref, it_ref, mg = oracle.mimo_plants_step(sh, Ad, Bd, X, U, N, nthreads=8, margins=True)
    assert np.all(st == sm.SOLVED)
    _check(x, st, it, Us[0], x_ref, st_ref, it_ref, U_ref, mg)


def test_siso_specialisation_matches_reference_controller(plant):
    """n_u = n_y = 1, K0 = K(0), w0 = 255, S rows = 10: the reference controller (config 3 plants)."""
    N, B = 20, 32
    rng = np.random.default_rng(5)
    Ad = plant["Ad"][None] * (1 + 0.02 * rng.normal(size=(B, 4, 4)))
    Bd = (plant["Bd"][None] * (1 + 0.02 * rng.normal(size=(B, 4))))[:, :, None]
    sh = {"Cd": plant["Cd"][None, :], "Q": [[plant["Q"]]], "R": [[plant["R"]]], "RD": [[plant["RD"]]],
          "K": plant["K"][None, :], "K0": [[plant["K"][0]]], "w0": [255.0]}
    X, U = workload.mpc_states(3, 0, B)
    Us, x, st, it = _run_device(sh, Ad, Bd, X, U[:, None], N, s_rows=10)
    U_ref, st_ref, it_ref = oracle.plants_step(plant, Ad, Bd[:, :, 0], X, U, N)
    _, x_ref, st2, it2, mg = oracle.mimo_plants_step(sh, Ad, Bd, X, U[:, None], N, s_rows=10, margins=True)
    assert np.array_equal(st_ref, st2) and np.array_equal(it_ref, it2)  # the two oracles agree
    _check(x, st, it, Us[0][:, 0], x_ref, st_ref, it_ref, U_ref, mg)


def test_random_mimo_with_state_bounds_and_reference():
    """n_x 3, n_u 2, n_y 2, N 8 with a state term in the bounds (K != 0, s_rows 5) and yref != 0."""
    N, B, nx, nu, ny = 8, 40, 3, 2, 2
    rng = np.random.default_rng(11)
    Ad = np.empty((B, nx, nx))
    for b in range(B):
        M = rng.normal(size=(nx, nx))
        Ad[b] = 0.9 * M / np.abs(np.linalg.eigvals(M)).max()
    Bd = rng.normal(size=(B, nx, nu))
    sh = {"Cd": rng.normal(size=(ny, nx)), "Q": np.diag([2.0, 0.5]), "R": np.diag([0.3, 0.1]),
          "RD": np.array([[1.0, 0.2], [0.2, 0.8]]), "K": 0.5 * rng.normal(size=(nu, nx)),
          "K0": np.array([[1.0, 0.3], [0.0, 0.8]]), "w0": np.array([0.8, 1.2])}
    X = rng.normal(size=(B, nx))
    U = 0.2 * rng.normal(size=(B, nu))
    yref = np.array([0.3, -0.2])
    Us, x, st, it = _run_device(sh, Ad, Bd, X, U, N, s_rows=5, yref=yref)
    U_ref, x_ref, st_ref, it_ref, mg = oracle.mimo_plants_step(sh, Ad, Bd, X, U, N, yref=yref, s_rows=5, margins=True)
    _check(x, st, it, Us[0], x_ref, st_ref, it_ref, U_ref, mg)


def test_second_step_is_warm_started():
    """A second controllerStep on the same context warm-starts from the first (:52) and matches an
    oracle solver that keeps its state across the two steps."""
    N, B = 30, 8
    Ad, Bd = workload.quadrotor_plants(3, 100, B)
    sh = workload.quadrotor_shared()
    X, U = workload.quadrotor_states(3, 100, B)
    Us, x, st, it = _run_device(sh, Ad, Bd, X, U, N, steps=2)
    for b in range(B):
        ops = oracle.condense_mimo(dict(sh, Ad=Ad[b], Bd=Bd[b]), N)
        n, m = ops["P"].shape[0], ops["A"].shape[0]
        r = oracle.Solver(ops["P"], np.zeros(n), ops["A"], np.full(m, -np.finfo(float).max), ops["W0"])
        u_cur = U[b].copy()
        for k in range(2):
            assert r.update_gradient(oracle.mimo_gradient(ops, X[b], u_cur))
            assert r.update_upper_bound(oracle.mimo_upper_bound(ops, X[b], u_cur))
            if r.solve() == oracle.SOLVED:
                u_cur = u_cur + r.x()[:4]
            np.testing.assert_allclose(Us[k][b], u_cur, rtol=0, atol=1e-7)
        assert st[b] == r.info().status


@pytest.mark.parametrize("over", [dict(max_iter=15), dict(adaptive_rho=0), dict(check_termination=5),
                                  dict(eps_abs=1e-5, eps_rel=1e-5), dict(scaling=0), dict(alpha=1.0, rho=1.0)],
                         ids=["max_iter", "no_adapt", "check5", "tight", "unscaled", "alpha1_rho1"])
def test_settings_variants_match_oracle(over):
    """OSQP settings the reference could set (osqp-eigen settings(), :51-52) on the quad-rotor batch:
    statuses (MAX_ITER_REACHED / SOLVED_INACCURATE included), iteration schedule and solutions."""
    N, B = 30, 16
    Ad, Bd = workload.quadrotor_plants(7, 0, B)
    sh = workload.quadrotor_shared()
    X, U = workload.quadrotor_states(7, 0, B)
    Us, x, st, it = _run_device(sh, Ad, Bd, X, U, N, settings=sm.default_settings(**over))
    U_ref, x_ref, st_ref, it_ref, mg = oracle.mimo_plants_step(sh, Ad, Bd, X, U, N,
                                                               settings=oracle.default_settings(**over),
                                                               nthreads=8, margins=True)
    _check(x, st, it, Us[0], x_ref, st_ref, it_ref, U_ref, mg)


def test_general_k0_path_on_diagonal_k0(monkeypatch):
    """The exchange path (general K0) run on the quad-rotor (diagonal K0) gives the oracle's results too."""
    monkeypatch.setenv("MPCQ_MIMO_GENERAL_K0", "1")
    N, B = 30, 12
    Ad, Bd = workload.quadrotor_plants(9, 0, B)
    sh = workload.quadrotor_shared()
    X, U = workload.quadrotor_states(9, 0, B)
    Us, x, st, it = _run_device(sh, Ad, Bd, X, U, N)
    U_ref, x_ref, st_ref, it_ref, mg = oracle.mimo_plants_step(sh, Ad, Bd, X, U, N, nthreads=8, margins=True)
    _check(x, st, it, Us[0], x_ref, st_ref, it_ref, U_ref, mg)


def test_nonconvex_plant_fails_setup():
    """A plant whose condensed Hessian has a negative diagonal (R < 0 beyond the tracking term) is
    rejected at setup, as osqp_setup rejects a non-convex P (the reference's ctor: solverFlag false),
    instead of surfacing later as a per-QP NON_CVX status."""
    N, B = 30, 4
    Ad, Bd = workload.quadrotor_plants(3, 0, B)
    sh = dict(workload.quadrotor_shared())
    sh["R"] = -1e6 * np.eye(4)
    X, U = workload.quadrotor_states(3, 0, B)
    with pytest.raises(sm.MpcqError, match="not positive definite"):
        _run_device(sh, Ad, Bd, X, U, N)


def test_quadrotor_bench_sample_matches_oracle():
    """4,096 plants of the config-4 bench batch (seed 3, its first plants; the oracle does ~500 of these
    per second per host share, so the full 262,144 are out of reach here) under the module's bar."""
    N, B = 30, 4096
    Ad, Bd = workload.quadrotor_plants(3, 0, B)
    sh = workload.quadrotor_shared()
    X, U = workload.quadrotor_states(3, 0, B)
    Us, x, st, it = _run_device(sh, Ad, Bd, X, U, N)
    U_ref, x_ref, st_ref, it_ref, mg = oracle.mimo_plants_step(sh, Ad, Bd, X, U, N, margins=True)
    assert np.all(st == sm.SOLVED)
    _check(x, st, it, Us[0], x_ref, st_ref, it_ref, U_ref, mg)
