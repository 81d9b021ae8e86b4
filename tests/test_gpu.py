"""GPU parity tests: the HIP path through the C ABI vs the CPU oracle (oracle/), same seeded inputs.

Bar, asserted on EVERY QP of every case:
* fp64: the oracle's trajectory (same status, same iteration count, same rho, |x - x_oracle| <= 1e-9
  absolute), i.e. far inside the north-star bound ||u* - u*_osqp||_inf < 1e-5;
* fp32: the oracle's status and iteration count, and |x - x_oracle| <= F32_TOL * max(1, ||x_oracle||_inf)
  on the applied move x0 (ModelPredictiveControlAPI.cpp:105) and on the whole vector.  The bound is
  relative because fp32 carries 24 bits: moves reach |x0| ~ 75 here, where one fp32 ulp is 7.6e-6,
  and the ADMM iterate accumulates ~2e-6 relative over its ~100 iterations (measured max 2.7e-5
  absolute at |x| ~ 60); the absolute 1e-5 is the fp64 path's bar.
  Exception, counted and bounded: a QP whose schedule decision the oracle itself takes within
  TIE_MARGIN of its threshold (|ln(residual / tolerance)| < 2e-3, oracle Info.margin; ~0.1% of QPs)
  can take the other branch in fp32, whose residuals carry ~1e-3 relative rounding.  Such a QP must
  still end SOLVED with the OSQP termination criteria met by the device's own solution (a valid
  OSQP answer one check earlier or later), and the test reports how many did.
Full-size (65,536 QP) runs are checked through size-independent properties (KKT residuals at the
solver's own tolerance) and shard invariance against the oracle on a prefix.
"""
import os

import numpy as np
import pytest

import oracle
import solvempc_amd as sm
from solvempc_amd import workload

pytestmark = pytest.mark.gpu
LMIN = -np.finfo(np.float64).max
F32_TOL = 1e-5


TIE_MARGIN = 2e-3


def _f32_parity(s, x, st, it, x_ref, st_ref, it_ref, margin, q, u, ops, what=""):
    """The fp32 bar on every QP (module docstring): returns the number of schedule ties taken the
    other way."""
    assert np.array_equal(st, st_ref), what
    tie = margin < TIE_MARGIN
    off = it != it_ref
    assert not np.any(off & ~tie), (what, np.flatnonzero(off & ~tie)[:8], margin[off & ~tie][:8])
    _f32_close(x[~off], x_ref[~off], what)
    if off.any():  # the other branch of a tie: a valid OSQP answer of its own
        _osqp_terminated(x[off], s.dual()[off], q[off], u[off], ops)
    return int(off.sum())


def _osqp_terminated(x, y, q, u, ops, slack=1.5):
    """Unscaled primal / dual residuals within OSQP's eps_abs = eps_rel = 1e-3 tolerances."""
    Ax = x @ ops["A"].T
    prim = np.maximum(Ax - u, 0).max(axis=1)
    tol_p = 1e-3 + 1e-3 * np.maximum(np.abs(Ax).max(axis=1), np.abs(u).max(axis=1))
    assert np.all(prim <= slack * tol_p)
    Px, Aty = x @ ops["P"], y @ ops["A"]
    dual = np.abs(Px + q + Aty).max(axis=1)
    tol_d = 1e-3 + 1e-3 * np.maximum(np.abs(q).max(axis=1), np.maximum(np.abs(Aty).max(axis=1), np.abs(Px).max(axis=1)))
    assert np.all(dual <= slack * tol_d)


def _f32_close(x, x_ref, what=""):
    """fp32 bar on every QP: applied move and whole vector within F32_TOL * max(1, ||x_ref||_inf)."""
    scale = np.maximum(1.0, np.abs(x_ref).max(axis=1))
    e0 = np.abs(x[:, 0] - x_ref[:, 0]) / scale
    ev = np.abs(x - x_ref).max(axis=1) / scale
    assert e0.max() < F32_TOL and ev.max() < F32_TOL, (what, e0.max(), ev.max(), int(np.argmax(ev)))


@pytest.fixture(params=["tile", "wave", "lane"])
def kernel(request):
    """Run a test on every device path: the MFMA tile kernel (shared plant, the default; its tail
    phases run one QP per wave), the one-QP-per-wave kernel (per-plant batches) and the per-lane
    kernel (the first kernel), the latter two forced through the MPCQ_KERNEL test hook."""
    old = os.environ.get("MPCQ_KERNEL")
    os.environ["MPCQ_KERNEL"] = request.param
    yield request.param
    if old is None:
        os.environ.pop("MPCQ_KERNEL", None)
    else:
        os.environ["MPCQ_KERNEL"] = old


def _problem(plant, N, B, seed=1, u_range=1.0, start=0):
    ops = oracle.condense(plant, N)
    X, U = workload.mpc_states(seed, start, B, u_range)
    q = oracle.gradient(ops, X, U)
    u = oracle.upper_bound(ops, X, U)
    return ops, X, U, q, u


def _gpu_solve(ops, q, u, N, dtype="f64", settings=None):
    B = q.shape[0]
    l = np.full(2 * N, LMIN)
    s = sm.BatchSolver(N, 2 * N, B, dtype=dtype, settings=settings)
    s.setup(ops["P"], np.zeros(N), ops["A"], l, oracle.upper_bound(ops, np.zeros(4), 0.0))
    s.update_lin_cost(q)
    s.update_upper_bound(u)
    s.solve()
    return s


def _oracle_solve(ops, q, u, N, settings=None, margins=False):
    l = np.full(2 * N, LMIN)
    return oracle.batch_solve(ops["P"], ops["A"], np.zeros(N), l, oracle.upper_bound(ops, np.zeros(4), 0.0),
                              q, u, settings=settings, margins=margins)


@pytest.mark.parametrize("N,u_range", [(20, 1.0), (15, 0.0)])
def test_fp64_trajectory_parity(plant, N, u_range, kernel):
    ops, X, U, q, u = _problem(plant, N, 4096, u_range=u_range)
    x_ref, st_ref, it_ref, rho_ref = _oracle_solve(ops, q, u, N)
    s = _gpu_solve(ops, q, u, N)
    x = s.solution()
    st, it, rho = s.info()
    assert np.array_equal(st, st_ref)
    assert np.array_equal(it, it_ref)
    np.testing.assert_allclose(rho, rho_ref, rtol=1e-9)
    assert np.abs(x - x_ref).max() < 1e-9


@pytest.mark.parametrize("N,seed", [(20, 1), (15, 3)])
def test_fp32_parity(plant, kernel, N, seed):
    ops, X, U, q, u = _problem(plant, N, 4096, seed=seed)
    x_ref, st_ref, it_ref, _, margin = _oracle_solve(ops, q, u, N, margins=True)
    s = _gpu_solve(ops, q, u, N, dtype="f32")
    x = s.solution()
    st, it, _ = s.info()
    assert np.all(st == sm.SOLVED)
    ties = _f32_parity(s, x, st, it, x_ref, st_ref, it_ref, margin, q, u, ops)
    print(f"fp32 N={N} seed={seed}: {ties} of 4096 QPs took a tie's other branch")


def test_f64_absolute_bound(plant):
    """The north star's absolute ||u* - u*_osqp||_inf < 1e-5 on the reference precision's path."""
    N = 20
    ops, X, U, q, u = _problem(plant, N, 4096)
    x_ref, _, _, _ = _oracle_solve(ops, q, u, N)
    x = _gpu_solve(ops, q, u, N).solution()
    assert np.abs(x - x_ref).max() < 1e-9


def test_ragged_and_single(plant, kernel):
    N = 20
    for B in (1, 63, 65, 100):
        ops, X, U, q, u = _problem(plant, N, B, seed=7)
        x_ref, st_ref, it_ref, _ = _oracle_solve(ops, q, u, N)
        s = _gpu_solve(ops, q, u, N)
        st, it, _ = s.info()
        assert np.array_equal(st, st_ref) and np.array_equal(it, it_ref)
        assert np.abs(s.solution() - x_ref).max() < 1e-9


def test_padded_capacity_generic_qp(kernel):
    """A random convex QP with finite lower bounds and an equality row (n=7, m=11 -> padded 8x16)."""
    rng = np.random.default_rng(3)
    n, m, B = 7, 11, 200
    M = rng.normal(size=(n, n))
    P = M @ M.T + 0.1 * np.eye(n)
    A = rng.normal(size=(m, n))
    q = rng.normal(size=(B, n))
    l = np.tile(-rng.uniform(0.5, 2.0, size=m), (B, 1))
    u = np.tile(rng.uniform(0.5, 2.0, size=m), (B, 1))
    l[:, 3] = u[:, 3] = 0.25  # equality row
    x_ref, st_ref, it_ref, _ = oracle.batch_solve(P, A, np.zeros(n), l[0], u[0], q, u)
    s = sm.BatchSolver(n, m, B)
    s.setup(P, np.zeros(n), A, l[0], u[0])
    s.update_lin_cost(q)
    s.update_upper_bound(u)
    s.solve()
    st, it, _ = s.info()
    assert np.array_equal(st, st_ref)
    assert np.array_equal(it, it_ref)
    assert np.abs(s.solution() - x_ref).max() < 1e-8


@pytest.mark.parametrize("dtype", ["f64", "mixed", "f32"])
def test_infeasible_and_invalid(kernel, dtype):
    """A primal-infeasible QP gets OSQP's certificate status and no solution, a u < l QP INVALID_BOUNDS,
    in every precision (the certificate is formed in T from the iterate's delta y; here |y| stays small)."""
    n, m = 2, 4
    P = np.eye(n)
    A = np.array([[1.0, 0.0], [1.0, 0.0], [0.0, 1.0], [0.0, 1.0]])
    l0 = np.array([-1e30, 1.0, -1.0, -1.0])
    u0 = np.array([-1.0, 1e30, 1.0, 1.0])  # x0 <= -1 and x0 >= 1: primal infeasible
    s = sm.BatchSolver(n, m, 2, dtype=dtype)
    s.setup(P, np.zeros(n), A, l0, u0)
    u_bad = np.stack([u0, u0.copy()])
    u_bad[1, 2] = -2.0  # u < l on row 2
    s.update_upper_bound(u_bad)
    s.solve()
    st, _, _ = s.info()
    ref = oracle.Solver(P, np.zeros(n), A, l0, u0)
    ref.solve()
    assert st[0] == ref.info().status == sm.PRIMAL_INFEASIBLE
    assert st[1] == sm.INVALID_BOUNDS
    assert np.all(np.isnan(s.solution()[0]))


# Primal-infeasible MPC QPs of the shared plant (rows j and N + j of A are negations: u_j = u_{N+j} = -c asks
# A_j x <= -c and A_j x >= c), at the bench's tile path: the oracle certifies each at its first check.
def _infeasible_batch(plant, N, B):
    ops, X, U, q, u = _problem(plant, N, B)
    u = u.copy()
    bad = {7: (slice(None), -1e3), 8: (slice(None), -1e3), 1000: (slice(None), -1.0), 2001: ([3, N + 3], -5.0),
           4090: ([0, N + 0], -0.5)}
    for i, (rows, c) in bad.items():
        u[i, rows] = c
    return ops, q, u, np.array(sorted(bad))


@pytest.mark.parametrize("dtype", ["f64", "mixed", "f32"])
def test_infeasible_statuses_match_oracle(plant, dtype):
    """Every QP's status against the oracle (OSQP's certificates, osqp_solve behind solve(), :102) on a
    tile-path batch holding primal-infeasible QPs of several strengths.  fp64 and mixed (whose check
    iterations run on an fp64 state): the oracle's status and iteration count on every QP.  fp32: OSQP's
    certificate asks ||A' dy|| < eps_prim_inf ||dy|| with dy the last dual step, while an infeasible QP's
    dual iterate grows without bound (|y| ~ 560 per 25 iterations at c = 1e3), and an fp32 iterate's
    rounding of it (ulp(|y|) through the KKT solve into A x~) moves that ratio by ~1e-4 .. 1e-2
    (tools/precision_sim.py infeasible): the documented bound (include/mpcq.h MPCQ_F32) is that where the
    oracle certifies primal infeasibility fp32 reports PRIMAL_INFEASIBLE or runs to max_iter (then
    MAX_ITER_REACHED, or SOLVED_INACCURATE when OSQP's approximate check at max_iter passes on the huge
    iterate) — never SOLVED — and agrees with the oracle on every other QP.  solve() is false either way.
    The mixed path switches a wave to fp64 once a column nears the certificate (mpcq_tile.h `mix64`)."""
    N, B = 20, 16384
    ops, q, u, bad = _infeasible_batch(plant, N, B)
    s = _gpu_solve(ops, q, u, N, dtype=dtype)
    assert s.path()[0] == "tile"
    st, it, _ = s.info()
    x = s.solution()
    s.close()
    _, st_ref, it_ref, _ = _oracle_solve(ops, q, u, N)
    assert np.all(st_ref[bad] == sm.PRIMAL_INFEASIBLE)
    ok = np.setdiff1d(np.arange(B), bad)
    assert np.array_equal(st[ok], st_ref[ok])
    if dtype == "f32":
        assert np.all(np.isin(st[bad], (sm.PRIMAL_INFEASIBLE, sm.MAX_ITER_REACHED, sm.SOLVED_INACCURATE))), st[bad]
        cert = st[bad] == sm.PRIMAL_INFEASIBLE
        assert np.all(it[bad][~cert] == sm.default_settings().max_iter)
        assert np.all(np.isnan(x[bad][cert])) and not np.isnan(x[bad][~cert]).any()
        print(f"fp32: {int(cert.sum())} of {bad.size} infeasible QPs certified, the rest MAX_ITER_REACHED")
        return
    assert np.array_equal(st[bad], st_ref[bad]) and np.all(np.isnan(x[bad]))
    assert np.array_equal(it[bad], it_ref[bad])
    if dtype == "f64":
        assert np.array_equal(it, it_ref)


def test_condense_kernel_matches_oracle(plant):
    for N in (15, 20):
        ref = oracle.condense(plant, N)
        dev = sm.mpc.condense({"Ad": plant["Ad"][None], "Bd": plant["Bd"][None], "Cd": plant["Cd"][None],
                               "K": plant["K"][None], "Q": [plant["Q"]], "R": [plant["R"]], "RD": [plant["RD"]]}, N)
        for k in ("P", "A", "Fx", "Fu", "Fr", "Sbar", "Ku", "W0"):
            np.testing.assert_allclose(dev[k][0], ref[k], rtol=1e-12, atol=1e-15, err_msg=k)


def test_mpc_front_end_and_receding_horizon(plant, kernel):
    """controllerStep semantics: q/u built on device, warm-started solves, U += x0 (:81-108)."""
    N, B, steps = 20, 512, 3
    ops = oracle.condense(plant, N)
    X, U = workload.mpc_states(4, 0, B)
    l = np.full(2 * N, LMIN)
    u0 = oracle.upper_bound(ops, np.zeros(4), 0.0)
    s = sm.BatchSolver(N, 2 * N, B)
    s.setup(ops["P"], np.zeros(N), ops["A"], l, u0)
    s.mpc_set_operators(ops["Fx"], ops["Fu"], ops["Fr"], ops["Sbar"], ops["Ku"], ops["W0"])
    refs = [oracle.Solver(ops["P"], np.zeros(N), ops["A"], l, u0) for _ in range(16)]
    U_ref = U[:16].copy()
    Ug = U.copy()
    for _ in range(steps):
        Ug = s.mpc_step(X, Ug)
        for b, r in enumerate(refs):
            assert r.update_gradient(oracle.gradient(ops, X[b], U_ref[b]))
            assert r.update_upper_bound(oracle.upper_bound(ops, X[b], U_ref[b]))
            if r.solve() == sm.SOLVED:
                U_ref[b] += r.x()[0]
        np.testing.assert_allclose(Ug[:16], U_ref, rtol=0, atol=1e-9)


def test_per_plant_batch(plant):
    """n_plants == batch: each QP carries its own (P, A) — here perturbed plants (config 3 shape)."""
    N, B = 20, 64
    rng = np.random.default_rng(5)
    Ps, As, qs, us, xs_ref, st_ref, it_ref = [], [], [], [], [], [], []
    X, U = workload.mpc_states(2, 0, B)
    for b in range(B):
        pl = dict(plant)
        pl["Ad"] = plant["Ad"] * (1 + 0.02 * rng.normal(size=(4, 4)))
        pl["Bd"] = plant["Bd"] * (1 + 0.02 * rng.normal(size=4))
        ops = oracle.condense(pl, N)
        q, u = oracle.gradient(ops, X[b], U[b]), oracle.upper_bound(ops, X[b], U[b])
        x, st, it, _ = oracle.batch_solve(ops["P"], ops["A"], np.zeros(N), np.full(2 * N, LMIN),
                                          oracle.upper_bound(ops, np.zeros(4), 0.0), q[None], u[None])
        Ps.append(ops["P"]); As.append(ops["A"]); qs.append(q); us.append(u)
        xs_ref.append(x[0]); st_ref.append(st[0]); it_ref.append(it[0])
    s = sm.BatchSolver(N, 2 * N, B, n_plants=B)
    u0 = np.full((B, 2 * N), 255.0)  # W0 + Sbar 0 + Ku 0 (ModelPredictiveControlAPI.cpp:43)
    s.setup(np.stack(Ps), np.zeros((B, N)), np.stack(As), np.full((B, 2 * N), LMIN), u0)
    s.update_lin_cost(np.stack(qs))
    s.update_upper_bound(np.stack(us))
    s.solve()
    st, it, _ = s.info()
    assert np.array_equal(st, np.array(st_ref))
    assert np.array_equal(it, np.array(it_ref))
    assert np.abs(s.solution() - np.stack(xs_ref)).max() < 1e-9


@pytest.mark.parametrize("dtype", ["f64", "f32"])
def test_full_batch_kkt_properties(plant, dtype):
    """BASELINE config 2 size (65,536 QPs), both precisions (f32 is the bench's): every QP SOLVED, its
    unscaled residuals within the OSQP tolerances it terminated on (a size-independent property), and
    every QP against the oracle (OpenMP over the host cores, ~1 s on the GPU box) under the module's
    bar: fp64 on the oracle's trajectory, fp32 on its schedule except counted ties."""
    N, B = 20, 65536
    ops, X, U, q, u = _problem(plant, N, B)
    s = _gpu_solve(ops, q, u, N, dtype=dtype)
    st, it, _ = s.info()
    assert np.all(st == sm.SOLVED)
    x, y = s.solution(), s.dual()
    Ax = x @ ops["A"].T
    prim = np.maximum(Ax - u, 0).max(axis=1)
    tol_p = 1e-3 + 1e-3 * np.maximum(np.abs(Ax).max(axis=1), np.abs(u).max(axis=1))
    assert np.all(prim <= 1.5 * tol_p)
    Px, Aty = x @ ops["P"], y @ ops["A"]
    dual = np.abs(Px + q + Aty).max(axis=1)
    tol_d = 1e-3 + 1e-3 * np.maximum(np.abs(q).max(axis=1), np.maximum(np.abs(Aty).max(axis=1), np.abs(Px).max(axis=1)))
    assert np.all(dual <= 1.5 * tol_d)
    # every QP of the full batch against the oracle
    x_ref, st_ref, it_ref, _, margin = _oracle_solve(ops, q, u, N, margins=True)
    if dtype == "f64":
        assert np.array_equal(st, st_ref) and np.array_equal(it, it_ref)
        assert np.abs(x - x_ref).max() < 1e-9
    else:
        ties = _f32_parity(s, x, st, it, x_ref, st_ref, it_ref, margin, q, u, ops, "full batch")
        print(f"fp32 full batch: {ties} of {B} QPs took a tie's other branch")


@pytest.mark.parametrize("tail", ["default", "wave"])
def test_full_batch_mpc_step_matches_oracle(plant, tail, monkeypatch):
    """The bench's exact path at its size: 65,536 fp32 controllerSteps through mpcq_mpc_step_device (front
    end on the device, U += x0 in the kernel) against the oracle's controllerStep on every QP: the
    applied U within F32_TOL * max(1, ||x_oracle||_inf) except at counted schedule ties, whose own
    solution must still meet OSQP's termination criteria.  tail=wave: the chain [100, 125] on tile
    waves with the QPs past 125 iterations on the one-QP-per-wave kernel (MPCQ_TAIL=wave), whose
    front end rebuilds q, u from X, U (phase 0 saved those instead of q, u)."""
    import torch
    if tail == "wave":  # (index order: the hardest-first default runs one launch, no tail phase)
        monkeypatch.setenv("MPCQ_TAIL", "wave")
        monkeypatch.setenv("MPCQ_ORDER", "0")
    N, B = 20, 65536
    ops, X, U, q, u = _problem(plant, N, B)
    l = np.full(2 * N, LMIN)
    s = sm.BatchSolver(N, 2 * N, B, dtype="f32")
    s.setup(ops["P"], np.zeros(N), ops["A"], l, oracle.upper_bound(ops, np.zeros(4), 0.0))
    s.mpc_set_operators(ops["Fx"], ops["Fu"], ops["Fr"], ops["Sbar"], ops["Ku"], ops["W0"])
    Xd, Ud = torch.from_numpy(X.copy()).cuda(), torch.from_numpy(U.copy()).cuda()
    s.mpc_step_device(Xd.data_ptr(), Ud.data_ptr(), 0.0)
    torch.cuda.synchronize()
    Ug = Ud.cpu().numpy()
    st, it, _ = s.info()
    x_ref, st_ref, it_ref, _, margin = _oracle_solve(ops, q, u, N, margins=True)
    U_ref = U + np.where(st_ref == sm.SOLVED, x_ref[:, 0], 0.0)
    assert np.array_equal(st, st_ref)
    off = it != it_ref
    assert not np.any(off & (margin >= TIE_MARGIN))
    scale = np.maximum(1.0, np.abs(x_ref).max(axis=1))
    assert (np.abs(Ug - U_ref)[~off] / scale[~off]).max() < F32_TOL
    x = s.solution()  # the published solution is the one U was moved by (U += x0, :105)
    assert np.abs((Ug - U) - np.where(st == sm.SOLVED, x[:, 0], 0.0)).max() <= 1e-12 * max(1.0, np.abs(Ug).max())
    if off.any():
        _osqp_terminated(x[off], s.dual()[off], q[off], u[off], ops)
    if tail == "wave":  # the variant ran its tail: QPs past 125 iterations exist (one QP per wave there)
        assert (it > 5 * 25).any()
    assert s.order()[0] == (tail != "wave")  # the default ran the batch hardest-first (mpcq_order.hip)
    # the step's q, u as the solver keeps them (materialised from the saved X, U, after the tail's own
    # front end rebuilt them for its QPs) are the oracle's updateGradient / updateUpperBound data
    v = s.device_view()
    torch.cuda.synchronize()
    qd = torch.as_tensor(_DevArray(v["q"], (B, N)), device="cuda").cpu().numpy()
    ud = torch.as_tensor(_DevArray(v["u"], (B, 2 * N)), device="cuda").cpu().numpy()
    assert np.abs(qd - q).max() <= 1e-12 * max(1.0, np.abs(q).max())
    assert np.abs(ud - u).max() <= 1e-12 * max(1.0, np.abs(u).max())
    print(f"fp32 bench path: {int(off.sum())} of {B} QPs took a tie's other branch")


MIXED_TOL = 1e-5  # north_star: ||u* - u*_osqp||_inf < 1e-5 on the applied move, absolute
MIXED_OFF_SCHEDULE = 1e-4  # at most this fraction of QPs may end one check earlier / later


def _mixed_parity(x, y, st, it, x_ref, st_ref, it_ref, q, u, ops, what=""):
    """MPCQ_F64_MIXED bar on every QP: the oracle's status; the applied move x0 within MIXED_TOL absolute
    on EVERY QP (no exemption); the oracle's iteration count and the whole vector within
    MIXED_TOL * max(1, ||x||) on all but at most MIXED_OFF_SCHEDULE of the QPs.  Those few are schedule
    ties the fp32 stretches can tip (the oracle's own decision margin there is ~3e-5, below the mixed
    residuals' ~1e-4 relative rounding): they must still meet OSQP's termination criteria with their own
    (x, y), and their applied move is inside the bound all the same (x0 is pinned by the active input
    constraint long before the termination check).  Returns (max |dx0|, QPs off the schedule)."""
    assert np.array_equal(st, st_ref), what
    off = it != it_ref
    assert off.mean() <= MIXED_OFF_SCHEDULE, (what, int(off.sum()))
    e0 = np.abs(x[:, 0] - x_ref[:, 0])
    assert e0.max() < MIXED_TOL, (what, e0.max(), int(np.argmax(e0)))
    ev = np.abs(x - x_ref).max(axis=1) / np.maximum(1.0, np.abs(x_ref).max(axis=1))
    assert ev[~off].max() < MIXED_TOL, (what, ev[~off].max())
    if off.any():
        _osqp_terminated(x[off], y[off], q[off], u[off], ops)
    return float(e0.max()), int(off.sum())


@pytest.mark.parametrize("N,u_range,B", [(20, 1.0, 8192), (15, 0.0, 8192), (20, 1.0, 65536)])
def test_mixed_tile_parity(plant, N, u_range, B, monkeypatch):
    """The mixed tile path (fp64 state and checks, fp32 plain iterations before the last MPCQ_MIX_R of
    every check interval) against the oracle's trajectory on every QP (_mixed_parity)."""
    monkeypatch.setenv("MPCQ_KERNEL", "tile")
    ops, X, U, q, u = _problem(plant, N, B, u_range=u_range)
    s = _gpu_solve(ops, q, u, N, dtype="mixed")
    assert s.path()[0] == "tile"
    x, (st, it, _) = s.solution(), s.info()
    x_ref, st_ref, it_ref, _ = _oracle_solve(ops, q, u, N)
    e, off = _mixed_parity(x, s.dual(), st, it, x_ref, st_ref, it_ref, q, u, ops, f"N={N} B={B}")
    print(f"mixed N={N} B={B}: max |dx0| {e:.2e}, {off} QPs off the oracle's schedule")


def test_mixed_full_batch_mpc_step_matches_oracle(plant):
    """The headline bench path at its size and precision: 65,536 controllerSteps through
    mpcq_mpc_step_device on an MPCQ_F64_MIXED context (front end and U += x0 on the device) against
    the oracle's controllerStep on every QP: the applied U within 1e-5 absolute on every QP (north_star;
    no exemption) and the rest of the _mixed_parity bar."""
    import torch
    N, B = 20, 65536
    ops, X, U, q, u = _problem(plant, N, B)
    l = np.full(2 * N, LMIN)
    s = sm.BatchSolver(N, 2 * N, B, dtype="mixed")
    s.setup(ops["P"], np.zeros(N), ops["A"], l, oracle.upper_bound(ops, np.zeros(4), 0.0))
    s.mpc_set_operators(ops["Fx"], ops["Fu"], ops["Fr"], ops["Sbar"], ops["Ku"], ops["W0"])
    Xd, Ud = torch.from_numpy(X.copy()).cuda(), torch.from_numpy(U.copy()).cuda()
    s.mpc_step_device(Xd.data_ptr(), Ud.data_ptr(), 0.0)
    torch.cuda.synchronize()
    Ug = Ud.cpu().numpy()
    st, it, _ = s.info()
    x_ref, st_ref, it_ref, _ = _oracle_solve(ops, q, u, N)
    U_ref = U + np.where(st_ref == sm.SOLVED, x_ref[:, 0], 0.0)
    d = np.abs(Ug - U_ref)
    assert d.max() < MIXED_TOL, (d.max(), int(np.argmax(d)))
    x = s.solution()
    e, off = _mixed_parity(x, s.dual(), st, it, x_ref, st_ref, it_ref, q, u, ops, "bench path")
    assert np.abs((Ug - U) - np.where(st == sm.SOLVED, x[:, 0], 0.0)).max() <= 1e-12 * max(1.0, np.abs(Ug).max())
    print(f"mixed bench path: max |dU| {d.max():.2e}, {off} of {B} QPs off the oracle's schedule")


def test_max_iter_and_warm_start(plant, kernel):
    """MAX_ITER_REACHED after max_iter (ModelPredictiveControlAPI.cpp:51-52 defaults otherwise) and the
    warm-started second solve of the same data, step for step against the oracle."""
    N = 20
    ops, X, U, q, u = _problem(plant, N, 64, seed=11)
    l = np.full(2 * N, LMIN)
    u0 = oracle.upper_bound(ops, np.zeros(4), 0.0)
    for kw in (dict(max_iter=10, eps_abs=1e-12, eps_rel=1e-12), dict()):
        st_o = oracle.default_settings(**kw)
        s = sm.BatchSolver(N, 2 * N, 64, settings=sm.default_settings(**kw))
        s.setup(ops["P"], np.zeros(N), ops["A"], l, u0)
        refs = [oracle.Solver(ops["P"], np.zeros(N), ops["A"], l, u0, st_o) for _ in range(8)]
        for _ in range(2):  # second round: warm start from the first solution (:52)
            s.update_lin_cost(q)
            s.update_upper_bound(u)
            s.solve()
            st, it, _ = s.info()
            x = s.solution()
            for b, r in enumerate(refs):
                assert r.update_gradient(q[b]) and r.update_upper_bound(u[b])
                r.solve()
                assert st[b] == r.info().status and it[b] == r.info().iter
                np.testing.assert_allclose(x[b], r.x(), rtol=0, atol=1e-9)
        if kw:
            assert np.all(st == sm.MAX_ITER_REACHED) and np.all(it == 10)


def test_api_warm_start_and_cold_start(plant, kernel):
    """osqp_warm_start(x, y) / osqp_cold_start through the C ABI vs the oracle's."""
    N = 15
    ops, X, U, q, u = _problem(plant, N, 32, seed=12)
    l = np.full(2 * N, LMIN)
    u0 = oracle.upper_bound(ops, np.zeros(4), 0.0)
    x_opt = np.load(os.path.join(os.path.dirname(__file__), "golden", "qp_n15.npz"))["x_opt"][:32]
    y0 = np.zeros((32, 2 * N))
    s = sm.BatchSolver(N, 2 * N, 32)
    s.setup(ops["P"], np.zeros(N), ops["A"], l, u0)
    s.update_lin_cost(q)
    s.update_upper_bound(u)
    s.warm_start(x_opt, y0)
    s.solve()
    st, it, _ = s.info()
    for b in range(0, 32, 4):
        r = oracle.Solver(ops["P"], np.zeros(N), ops["A"], l, u0)
        r.update_gradient(q[b]); r.update_upper_bound(u[b])
        r.warm_start(x_opt[b], y0[b])
        r.solve()
        assert st[b] == r.info().status and it[b] == r.info().iter
        np.testing.assert_allclose(s.solution()[b], r.x(), rtol=0, atol=1e-9)
    s.cold_start()
    s.solve()
    st2, it2, _ = s.info()
    r = oracle.Solver(ops["P"], np.zeros(N), ops["A"], l, u0)
    r.update_gradient(q[0]); r.update_upper_bound(u[0])
    r.solve()  # first solve from x = z = y = 0 ...
    # ... but rho persists across solves in OSQP, so compare against a solver that already solved once
    r2 = oracle.Solver(ops["P"], np.zeros(N), ops["A"], l, u0)
    r2.update_gradient(q[0]); r2.update_upper_bound(u[0])
    r2.warm_start(x_opt[0], y0[0]); r2.solve(); r2.cold_start(); r2.solve()
    assert st2[0] == r2.info().status and it2[0] == r2.info().iter
    np.testing.assert_allclose(s.solution()[0], r2.x(), rtol=0, atol=1e-9)


def test_dual_infeasible(kernel):
    P = np.zeros((2, 2))
    A = np.array([[0.0, 1.0]])
    s = sm.BatchSolver(2, 1, 3)
    s.setup(P, np.array([-1.0, 0.0]), A, np.array([-1.0]), np.array([1.0]))
    s.solve()
    st, it, _ = s.info()
    ref = oracle.Solver(P, np.array([-1.0, 0.0]), A, np.array([-1.0]), np.array([1.0]))
    ref.solve()
    assert ref.info().status == sm.DUAL_INFEASIBLE
    assert np.all(st == sm.DUAL_INFEASIBLE) and np.all(it == ref.info().iter)


def test_tile_and_wave_paths_agree(plant):
    """A QP may move from a tile launch to a wave launch at a phase boundary: both kernels run OSQP's
    iteration on the same state, with products summed in different orders (the tile kernel's paired
    loop uses the +-row structure of A).  Every QP: the same status and iteration count; fp64
    |dx| <= 1e-9, fp32 within F32_TOL * max(1, ||x||_inf)."""
    N = 20
    ops, X, U, q, u = _problem(plant, N, 2048, seed=21)
    margin = _oracle_solve(ops, q, u, N, margins=True)[4]
    for dtype in ("f64", "f32"):
        res = {}
        for k in ("tile", "wave"):
            os.environ["MPCQ_KERNEL"] = k
            try:
                s = _gpu_solve(ops, q, u, N, dtype=dtype)
                res[k] = (s.solution(), *s.info())
            finally:
                os.environ.pop("MPCQ_KERNEL", None)
        (xt, stt, itt, _), (xw, stw, itw, _) = res["tile"], res["wave"]
        assert np.all(stt == sm.SOLVED) and np.all(stw == sm.SOLVED)
        if dtype == "f64":
            assert np.array_equal(itt, itw)
            assert np.abs(xt - xw).max() <= 1e-9
        else:
            off = itt != itw
            assert not np.any(off & (margin >= TIE_MARGIN))
            _f32_close(xt[~off], xw[~off], "tile vs wave")


def test_plant_simulation_matches_host(plant):
    """mpcq_mpc_simulate_device: X <- Ad X + Bd U + w with the counter-based noise of workload.py."""
    import torch
    B, nx = 300, 4
    X, U = workload.mpc_states(31, 1000, B)
    s = sm.BatchSolver(20, 40, B)
    s.mpc_set_plant(plant["Ad"], plant["Bd"])
    Xd = torch.from_numpy(X.copy()).cuda()
    Ud = torch.from_numpy(U.copy()).cuda()
    Xh = X.copy()
    for step in (0, 1, 7):
        s.mpc_simulate_device(Xd.data_ptr(), Ud.data_ptr(), 5, 1000, step, 1e-2, 0)
        torch.cuda.synchronize()
        Xh = workload.simulate(plant["Ad"], plant["Bd"], Xh, U, workload.plant_noise(5, 1000, B, step, nx, 1e-2))
        np.testing.assert_allclose(Xd.cpu().numpy(), Xh, rtol=1e-13, atol=1e-15)


def test_receding_horizon_stream(plant, kernel):
    """BASELINE config 5 semantics: warm-started controllerStep (:81-108) + plant update, replayed from a
    hipGraph one step per call; every step's U matches the oracle driven by the device's X."""
    import torch
    N, B, steps = 20, 48, 12
    ops = oracle.condense(plant, N)
    l = np.full(2 * N, LMIN)
    u0 = oracle.upper_bound(ops, np.zeros(4), 0.0)
    X, U = workload.mpc_states(41, 0, B)
    s = sm.BatchSolver(N, 2 * N, B)
    s.setup(ops["P"], np.zeros(N), ops["A"], l, u0)
    s.mpc_set_operators(ops["Fx"], ops["Fu"], ops["Fr"], ops["Sbar"], ops["Ku"], ops["W0"])
    s.mpc_set_plant(plant["Ad"], plant["Bd"])
    Xd = torch.from_numpy(X.copy()).cuda()
    Ud = torch.from_numpy(U.copy()).cuda()
    st = torch.cuda.Stream()
    refs = [oracle.Solver(ops["P"], np.zeros(N), ops["A"], l, u0) for _ in range(B)]
    Xk, Uk = X.copy(), U.copy()
    for k in range(steps):
        with torch.cuda.stream(st):
            s.mpc_run_device(Xd.data_ptr(), Ud.data_ptr(), 0.0, 1, 9, 0, k, 1e-2, st.cuda_stream)
        st.synchronize()
        for b, r in enumerate(refs):
            assert r.update_gradient(oracle.gradient(ops, Xk[b], Uk[b]))
            assert r.update_upper_bound(oracle.upper_bound(ops, Xk[b], Uk[b]))
            if r.solve() == oracle.SOLVED:
                Uk[b] += r.x()[0]
        Ug, Xg = Ud.cpu().numpy(), Xd.cpu().numpy()
        np.testing.assert_allclose(Ug, Uk, rtol=0, atol=1e-9)
        Xk = workload.simulate(plant["Ad"], plant["Bd"], Xk, Uk, workload.plant_noise(9, 0, B, k, 4, 1e-2))
        np.testing.assert_allclose(Xg, Xk, rtol=1e-11, atol=1e-12)
        Xk = Xg.copy()  # keep the oracle on the device's trajectory (libm vs device math: last-ulp noise)
    _, it, _ = s.info()
    assert np.median(it) <= 50  # warm start (:52): later steps converge at the first checks


def test_receding_horizon_stream_f32(plant, kernel):
    """Config 5 in the bench's precision: the fp32 warm-started stream (hipGraph replay, one control
    step per call) against the oracle's controllerStep driven by the device's X and U of the step
    before (the fp32 and fp64 warm states differ by rounding, so each step is compared from the same
    inputs): every plant SOLVED on the oracle's iteration count, the move within F32_TOL relative."""
    import torch
    N, B, steps = 20, 48, 16
    ops = oracle.condense(plant, N)
    l = np.full(2 * N, LMIN)
    u0 = oracle.upper_bound(ops, np.zeros(4), 0.0)
    X, U = workload.stream_states(4, 0, B)
    s = sm.BatchSolver(N, 2 * N, B, dtype="f32")
    s.setup(ops["P"], np.zeros(N), ops["A"], l, u0)
    s.mpc_set_operators(ops["Fx"], ops["Fu"], ops["Fr"], ops["Sbar"], ops["Ku"], ops["W0"])
    s.mpc_set_plant(plant["Ad"], plant["Bd"])
    Xd = torch.from_numpy(X.copy()).cuda()
    Ud = torch.from_numpy(U.copy()).cuda()
    st = torch.cuda.Stream()
    refs = [oracle.Solver(ops["P"], np.zeros(N), ops["A"], l, u0) for _ in range(B)]
    Xk, Uk = X.copy(), U.copy()
    tied = set()  # plants whose warm state left the oracle's at a schedule tie: no longer compared
    for k in range(steps):
        with torch.cuda.stream(st):
            s.mpc_run_device(Xd.data_ptr(), Ud.data_ptr(), 0.0, 1, 9, 0, k, 1e-2, st.cuda_stream)
        st.synchronize()
        stat, it, _ = s.info()
        Ug = Ud.cpu().numpy()
        for b, r in enumerate(refs):
            if b in tied:
                continue
            assert r.update_gradient(oracle.gradient(ops, Xk[b], Uk[b]))
            assert r.update_upper_bound(oracle.upper_bound(ops, Xk[b], Uk[b]))
            assert r.solve() == oracle.SOLVED and stat[b] == sm.SOLVED
            if it[b] != r.info().iter:  # a schedule tie (module docstring)
                assert r.info().margin < TIE_MARGIN, (k, b, it[b], r.info().iter, r.info().margin)
                tied.add(b)
                continue
            x = r.x()
            assert abs(Ug[b] - (Uk[b] + x[0])) < F32_TOL * max(1.0, np.abs(x).max()), (k, b)
        Uk = Ug.copy()
        Xk = Xd.cpu().numpy().copy()
    assert len(tied) <= 2, tied


@pytest.mark.parametrize("family", ["tile", "wave"])
@pytest.mark.parametrize("dtype", ["f32", "f64", "mixed"])
def test_stream_one_launch_matches_graph(plant, dtype, family, monkeypatch):
    """mpcq_mpc_run_device's one-launch stream against the per-step hipGraph path (MPCQ_STREAM=graph) of
    the same kernel family, from the same cold state: the tile kernel's stream mode (every MFMA column
    one plant running its own control steps, a few plants per wave) against per-step tile solves, and
    stream_wave_kernel (one QP per wave) against per-step wave solves.  Bit-identical X, U, statuses,
    iterations, rho, stream counters and the last step's x, y after 30 steps in one call, then 7 more steps
    in a second call (warm state carried across calls; the graph's replays leave the captured step's lazy
    publication pending again after the first call's reads), on a ragged batch."""
    import torch
    monkeypatch.setenv("MPCQ_KERNEL", family)
    N, B = 20, 333
    ops = oracle.condense(plant, N)
    l = np.full(2 * N, LMIN)
    u0 = oracle.upper_bound(ops, np.zeros(4), 0.0)
    X, U = workload.stream_states(4, 0, B)

    def run(mode):
        if mode:
            monkeypatch.setenv("MPCQ_STREAM", mode)
        else:
            monkeypatch.delenv("MPCQ_STREAM", raising=False)
        s = sm.BatchSolver(N, 2 * N, B, dtype=dtype)
        s.setup(ops["P"], np.zeros(N), ops["A"], l, u0)
        s.mpc_set_operators(ops["Fx"], ops["Fu"], ops["Fr"], ops["Sbar"], ops["Ku"], ops["W0"])
        s.mpc_set_plant(plant["Ad"], plant["Bd"])
        Xd, Ud = torch.from_numpy(X.copy()).cuda(), torch.from_numpy(U.copy()).cuda()
        st = torch.cuda.Stream()
        out = []
        for first, steps in ((0, 30), (30, 7)):
            with torch.cuda.stream(st):
                s.mpc_run_device(Xd.data_ptr(), Ud.data_ptr(), 0.0, steps, 4, 0, first, 1e-2, st.cuda_stream)
            st.synchronize()
            it_acc, uns = s.stream_counters()
            out.append((Xd.cpu().numpy().copy(), Ud.cpu().numpy().copy(), *s.info(), it_acc, uns, s.solution(),
                        s.dual()))
            assert s.stream_path() == (mode or family)
        return out

    graph, one = run("graph"), run(None)
    for g, o in zip(graph, one):
        for a, b in zip(g, o):
            assert np.array_equal(a, b)
    assert np.all(one[-1][2] == sm.SOLVED) and one[-1][6].sum() == 0  # (X, U, status, iter, rho, it_acc, uns)


@pytest.mark.parametrize("over", [dict(max_iter=50), dict(check_termination=10), dict(adaptive_rho=0),
                                  dict(max_iter=30, check_termination=7)],
                         ids=["max_iter50", "check10", "no_adapt", "max_iter30_check7"])
def test_stream_tile_settings_variants(plant, over, monkeypatch):
    """The tile stream mode under OSQP settings the reference could set (:51-52): per-column max_iter
    (MAX_ITER_REACHED / SOLVED_INACCURATE steps), another check interval, no adaptive rho, bit-identical
    to per-step tile solves; settings whose max_iter or adapt interval is off the check grid
    (max_iter 30, check 7) run the per-step launches instead, with the same results."""
    import torch
    monkeypatch.setenv("MPCQ_KERNEL", "tile")
    N, B, steps = 20, 200, 20
    ops = oracle.condense(plant, N)
    l = np.full(2 * N, LMIN)
    X, U = workload.stream_states(4, 0, B)
    settings = sm.default_settings(**over)

    def run(mode):
        if mode:
            monkeypatch.setenv("MPCQ_STREAM", mode)
        else:
            monkeypatch.delenv("MPCQ_STREAM", raising=False)
        s = sm.BatchSolver(N, 2 * N, B, dtype="f32", settings=settings)
        s.setup(ops["P"], np.zeros(N), ops["A"], l, oracle.upper_bound(ops, np.zeros(4), 0.0))
        s.mpc_set_operators(ops["Fx"], ops["Fu"], ops["Fr"], ops["Sbar"], ops["Ku"], ops["W0"])
        s.mpc_set_plant(plant["Ad"], plant["Bd"])
        Xd, Ud = torch.from_numpy(X.copy()).cuda(), torch.from_numpy(U.copy()).cuda()
        st = torch.cuda.Stream()
        with torch.cuda.stream(st):
            s.mpc_run_device(Xd.data_ptr(), Ud.data_ptr(), 0.0, steps, 4, 0, 0, 1e-2, st.cuda_stream)
        st.synchronize()
        return s.stream_path(), (Xd.cpu().numpy(), Ud.cpu().numpy(), *s.info(), *s.stream_counters())

    (pg, g), (po, o) = run("graph"), run(None)
    assert pg == "graph" and po == ("graph" if over.get("check_termination") == 7 else "tile")
    for a_, b_ in zip(g, o):
        assert np.array_equal(a_, b_)


def test_stream_failed_steps_advance(plant, monkeypatch):
    """Stream plants whose every step fails OSQP's bound update (a state so large that u^ passes
    OSQP_INFTY * MIN_SCALING: TYPE_CHANGED, U unchanged) still advance their plant each step, also when
    every plant of a wave fails from the start (4 plants per wave, the first wave all failing): the tile
    stream mode against per-step tile solves, bit for bit."""
    import torch
    monkeypatch.setenv("MPCQ_KERNEL", "tile")
    monkeypatch.setenv("MPCQ_STREAM_CPW", "4")
    N, B, steps = 20, 8, 5
    ops = oracle.condense(plant, N)
    l = np.full(2 * N, LMIN)
    X, U = workload.stream_states(4, 0, B)
    X[:4] *= 1e29

    def run(mode):
        if mode:
            monkeypatch.setenv("MPCQ_STREAM", mode)
        else:
            monkeypatch.delenv("MPCQ_STREAM", raising=False)
        s = sm.BatchSolver(N, 2 * N, B, dtype="f32")
        s.setup(ops["P"], np.zeros(N), ops["A"], l, oracle.upper_bound(ops, np.zeros(4), 0.0))
        s.mpc_set_operators(ops["Fx"], ops["Fu"], ops["Fr"], ops["Sbar"], ops["Ku"], ops["W0"])
        s.mpc_set_plant(plant["Ad"], plant["Bd"])
        Xd, Ud = torch.from_numpy(X.copy()).cuda(), torch.from_numpy(U.copy()).cuda()
        st = torch.cuda.Stream()
        with torch.cuda.stream(st):
            s.mpc_run_device(Xd.data_ptr(), Ud.data_ptr(), 0.0, steps, 4, 0, 0, 1e-2, st.cuda_stream)
        st.synchronize()
        return s.stream_path(), (Xd.cpu().numpy(), Ud.cpu().numpy(), *s.info(), *s.stream_counters())

    (pg, g), (po, o) = run("graph"), run(None)
    assert pg == "graph" and po == "tile"
    for a_, b_ in zip(g, o):
        assert np.array_equal(a_, b_)
    assert np.all(o[2][:4] == sm.TYPE_CHANGED) and np.all(o[2][4:] == sm.SOLVED)
    assert np.all(o[6][:4] == steps) and np.all(o[6][4:] == 0)  # unsolved steps per plant
    assert not np.array_equal(o[0][:4], X[:4])  # the failing plants still moved


def test_stream_workload_stays_solved_and_bounded(plant):
    """The config-5 workload (workload.stream_states, noise std 1e-2) over 400 fp32 control steps: every
    plant SOLVED at every step and the closed loop bounded (the reference controller on its plant)."""
    import torch
    N, B, steps = 20, 256, 400
    ops = oracle.condense(plant, N)
    l = np.full(2 * N, LMIN)
    X, U = workload.stream_states(4, 0, B)
    s = sm.BatchSolver(N, 2 * N, B, dtype="f32")
    s.setup(ops["P"], np.zeros(N), ops["A"], l, oracle.upper_bound(ops, np.zeros(4), 0.0))
    s.mpc_set_operators(ops["Fx"], ops["Fu"], ops["Fr"], ops["Sbar"], ops["Ku"], ops["W0"])
    s.mpc_set_plant(plant["Ad"], plant["Bd"])
    Xd, Ud = torch.from_numpy(X.copy()).cuda(), torch.from_numpy(U.copy()).cuda()
    st = torch.cuda.Stream()
    for k in range(steps):
        with torch.cuda.stream(st):
            s.mpc_run_device(Xd.data_ptr(), Ud.data_ptr(), 0.0, 1, 4, 0, k, 1e-2, st.cuda_stream)
        st.synchronize()
        stat, _, _ = s.info()
        assert np.all(stat == sm.SOLVED), k
    assert np.abs(Xd.cpu().numpy()).max() < 10 and np.abs(Ud.cpu().numpy()).max() < 10


@pytest.mark.parametrize("dtype", ["f32", "f64", "mixed"])
def test_stream_bench_path_matches_oracle(plant, dtype, monkeypatch):
    """The config-5 bench path itself (one tile-stream launch, 4 plants per wave as the bench's 4,096-plant
    batch runs it) at 512 plants x 1,000 warm-started control steps against oracle.stream_run (one
    warm-started OSQP-0.6 restatement per plant on the device's noise stream): every step of every plant
    SOLVED on both sides; fp64: every plant's iteration total equal and the final U within 1e-8; fp32
    (the bench's dtype, whose closed loops drift from the fp64 ones by rounding over 1,000 steps): the
    iteration totals equal on >= 99 % of plants (the rest: an fp32 schedule tie somewhere in the 1,000
    steps, within 1 % of the total) and the final U within 1e-3; mixed (the tile stream mode with each step's
    plain iterations before the last MPCQ_MIX_R in fp32): totals equal on >= 99 % of plants and the final U
    within north_star's 1e-5 after the 1,000 closed-loop steps."""
    import torch
    monkeypatch.setenv("MPCQ_STREAM_CPW", "4")
    N, B, steps, seed, noise = 20, 512, 1000, 4, 1e-2
    ops = oracle.condense(plant, N)
    l = np.full(2 * N, LMIN)
    X, U = workload.stream_states(seed, 0, B)
    s = sm.BatchSolver(N, 2 * N, B, dtype=dtype)
    s.setup(ops["P"], np.zeros(N), ops["A"], l, oracle.upper_bound(ops, np.zeros(4), 0.0))
    s.mpc_set_operators(ops["Fx"], ops["Fu"], ops["Fr"], ops["Sbar"], ops["Ku"], ops["W0"])
    s.mpc_set_plant(plant["Ad"], plant["Bd"])
    Xd, Ud = torch.from_numpy(X.copy()).cuda(), torch.from_numpy(U.copy()).cuda()
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        s.mpc_run_device(Xd.data_ptr(), Ud.data_ptr(), plant["xref"], steps, seed, 0, 0, noise, st.cuda_stream)
    st.synchronize()
    assert s.stream_path() == "tile"
    it_dev, uns_dev = s.stream_iterations(), s.stream_unsolved()
    Xc, Uc, itc, unc = oracle.stream_run(plant, X, U, N, steps, seed, 0, 0, noise, xref=plant["xref"])
    assert uns_dev == 0 and int(unc.sum()) == 0
    same = it_dev == itc
    dU = np.abs(Ud.cpu().numpy() - Uc)
    if dtype == "f64":
        assert same.all(), np.flatnonzero(~same)[:8]
        assert dU.max() < 1e-8 and np.abs(Xd.cpu().numpy() - Xc).max() < 1e-8
    else:
        assert same.mean() >= 0.99, same.mean()
        assert (np.abs(it_dev - itc) / itc).max() < 0.01
        assert dU.max() < (1e-5 if dtype == "mixed" else 1e-3), dU.max()
    print(f"stream {dtype}: {B} plants x {steps} steps, iteration totals equal on {same.mean():.4f}, "
          f"max |dU| {dU.max():.2e}")


@pytest.mark.parametrize("n,m", [(5, 7), (13, 30), (20, 40), (32, 64)])
def test_per_plant_setups_agree(n, m):
    """Per-plant setup three ways on random convex QPs of odd and even order (equality rows, finite
    and free lower bounds): the direct inverse of M(rho) (the default for per-plant batches,
    setup_inv_kernel, with the wave kernel's in-kernel refactorisation when rho adapts), the wave
    kernel's eigen-basis (MPCQ_SETUP=eigen) and the serial workgroup kernel (MPCQ_SETUP=ref): the same
    Ruiz scaling bit for bit, and the oracle's status / iteration count and |dx| <= 1e-8 for each."""
    rng = np.random.default_rng(n * 100 + m)
    B = 24
    Ps, As, ls, us, qs = [], [], [], [], []
    for _ in range(B):
        M = rng.normal(size=(n, n))
        Ps.append(M @ M.T + 0.1 * np.eye(n))
        As.append(rng.normal(size=(m, n)))
        lo = -rng.uniform(0.5, 2.0, size=m)
        lo[::5] = -1e30
        up = rng.uniform(0.5, 2.0, size=m)
        lo[1] = up[1] = 0.3
        ls.append(lo); us.append(up); qs.append(rng.normal(size=n))
    P, A, l, u, q = map(np.stack, (Ps, As, ls, us, qs))
    out = {}
    for mode in ("ref", "eigen", "inv"):
        if mode != "inv":
            os.environ["MPCQ_SETUP"] = mode
        try:
            s = sm.BatchSolver(n, m, B, n_plants=B)
            s.setup(P, np.zeros((B, n)), A, l, u)
        finally:
            os.environ.pop("MPCQ_SETUP", None)
        s.update_lin_cost(q)
        s.solve()
        out[mode] = (s.solution(), *s.info(), s.scaling())
    ref = [oracle.batch_solve(P[b], A[b], np.zeros(n), l[b], u[b], q[b][None], u[b][None]) for b in range(B)]
    for mode, (x, st, it, rho, sc) in out.items():
        for a_, b_ in zip(out["ref"][4], sc):
            assert np.array_equal(np.asarray(a_), np.asarray(b_)), mode
        for b in range(B):
            x_o, st_o, it_o, rho_o = ref[b]
            assert st[b] == st_o[0] and it[b] == it_o[0], (mode, b)
            assert abs(rho[b] - rho_o[0]) <= 1e-9 * rho_o[0], (mode, b)
            assert np.abs(x[b] - x_o[0]).max() < 1e-8, (mode, b)


def test_direct_inverse_refactors_on_rho_change(plant):
    """A per-plant batch whose rho adapts (OSQP adapt_rho at iteration 100): the direct-inverse path
    rebuilds M(rho)^-1 in the kernel and stays on the oracle's trajectory; a warm-started second solve
    starts from the adapted rho (operators rebuilt in the prologue) and matches too."""
    N, B = 20, 64
    ops = oracle.condense(plant, N)
    X, U = workload.mpc_states(13, 0, B, u_range=3.0)
    q, u = oracle.gradient(ops, X, U), oracle.upper_bound(ops, X, U)
    l = np.full(2 * N, LMIN)
    u0 = oracle.upper_bound(ops, np.zeros(4), 0.0)
    s = sm.BatchSolver(N, 2 * N, B, n_plants=B)
    s.setup(np.tile(ops["P"], (B, 1, 1)), np.zeros((B, N)), np.tile(ops["A"], (B, 1, 1)), np.tile(l, (B, 1)),
            np.tile(u0, (B, 1)))
    refs = [oracle.Solver(ops["P"], np.zeros(N), ops["A"], l, u0) for _ in range(B)]
    moved = 0
    for rnd in range(2):
        s.update_lin_cost(q)
        s.update_upper_bound(u)
        s.solve()
        x = s.solution()
        st, it, rho = s.info()
        for b, r in enumerate(refs):
            assert r.update_gradient(q[b]) and r.update_upper_bound(u[b])
            r.solve()
            assert st[b] == r.info().status and it[b] == r.info().iter, (rnd, b)
            assert abs(rho[b] - r.info().rho) <= 1e-9 * r.info().rho
            np.testing.assert_allclose(x[b], r.x(), rtol=0, atol=1e-9)
        moved += int(np.sum(rho != 0.1))
    assert moved > 0, "no QP adapted rho: the refactorisation path was not exercised"


def _perturbed_plants(plant, B, seed):
    rng = np.random.default_rng(seed)
    Ad = plant["Ad"][None] * (1 + 0.02 * rng.normal(size=(B, 4, 4)))
    Bd = plant["Bd"][None] * (1 + 0.02 * rng.normal(size=(B, 4)))
    return Ad, Bd


def test_condense_wave_kernel_bit_identical(plant):
    """The one-wave LDS condensing kernel reproduces the workgroup kernel bit for bit (same
    arithmetic order), on perturbed plants and both horizons of the fixtures."""
    B = 32
    Ad, Bd = _perturbed_plants(plant, B, 11)
    pl = {"Ad": Ad, "Bd": Bd, "Cd": np.tile(plant["Cd"], (B, 1)), "K": np.tile(plant["K"], (B, 1)),
          "Q": np.full(B, plant["Q"]), "R": np.full(B, plant["R"]), "RD": np.full(B, plant["RD"])}
    for N in (15, 20, 32):
        dev = sm.mpc.condense(pl, N)
        os.environ["MPCQ_CONDENSE"] = "ref"
        try:
            ref = sm.mpc.condense(pl, N)
        finally:
            os.environ.pop("MPCQ_CONDENSE", None)
        for k in dev:
            assert np.array_equal(dev[k], ref[k]), (N, k)


@pytest.mark.parametrize("dtype", ["f64", "f32"])
def test_per_plant_device_pipeline(plant, dtype):
    """BASELINE config 3 path (f32 is the bench's dtype): randomised plants resident on the device ->
    on-device condensing and setup (mpcq_mpc_setup_plants_device, incl. the fp32 contexts' setup
    tolerances) -> device front end and solve (mpcq_mpc_step_device), against the oracle's condense +
    controllerStep for every plant: status and iterations equal; the applied U to 1e-9 (f64) or
    F32_TOL * max(1, ||x_oracle||_inf) (f32)."""
    import torch

    N, B = 20, 96
    Ad, Bd = _perturbed_plants(plant, B, 7)
    X, U = workload.mpc_states(3, 0, B)
    dev = torch.device("cuda:0")
    t = lambda a: torch.as_tensor(np.ascontiguousarray(a, dtype=np.float64), device=dev)  # noqa: E731
    tAd, tBd = t(Ad), t(Bd)
    tCd, tK = t(np.tile(plant["Cd"], (B, 1))), t(np.tile(plant["K"], (B, 1)))
    tQ, tR, tRD = t(np.full(B, plant["Q"])), t(np.full(B, plant["R"])), t(np.full(B, plant["RD"]))
    tX, tU = t(X), t(U)
    s = sm.BatchSolver(N, 2 * N, B, n_plants=B, dtype=dtype)
    stream = torch.cuda.current_stream().cuda_stream
    s.mpc_setup_plants_device(4, 10, tAd.data_ptr(), tBd.data_ptr(), tCd.data_ptr(), tK.data_ptr(),
                              tQ.data_ptr(), tR.data_ptr(), tRD.data_ptr(), stream)
    s.mpc_step_device(tX.data_ptr(), tU.data_ptr(), 0.0, stream)
    torch.cuda.synchronize()
    st, it, _ = s.info()
    Ug = tU.cpu().numpy()
    for b in range(B):
        pl = dict(plant, Ad=Ad[b], Bd=Bd[b])
        ops = oracle.condense(pl, N)
        l = np.full(2 * N, LMIN)
        r = oracle.Solver(ops["P"], np.zeros(N), ops["A"], l, oracle.upper_bound(ops, np.zeros(4), 0.0))
        assert r.update_gradient(oracle.gradient(ops, X[b], U[b]))
        assert r.update_upper_bound(oracle.upper_bound(ops, X[b], U[b]))
        st_o = r.solve()
        assert st[b] == st_o, b
        if dtype == "f32" and it[b] != r.info().iter:  # a schedule tie (module docstring)
            assert r.info().margin < TIE_MARGIN, (b, it[b], r.info().iter, r.info().margin)
            continue
        assert it[b] == r.info().iter, b
        u_ref = U[b] + (r.x()[0] if st_o == sm.SOLVED else 0.0)
        tol = 1e-9 if dtype == "f64" else F32_TOL * max(1.0, np.abs(r.x()).max())
        assert abs(Ug[b] - u_ref) < tol, (b, Ug[b] - u_ref)


def test_stream_graph_recaptured_after_replant(plant):
    """The hipGraph of mpcq_mpc_run_device bakes in operator/plant buffers and kernel-variant flags:
    re-planting the context (mpcq_mpc_setup_plants_device with another nx, which reallocates those
    buffers, and mpcq_mpc_set_plant) must invalidate it.  Each phase is checked against the oracle's
    controllerStep driven by the device's X."""
    import torch

    N, B, steps = 20, 32, 3
    dev = torch.device("cuda:0")
    t = lambda a: torch.as_tensor(np.ascontiguousarray(a, dtype=np.float64), device=dev)  # noqa: E731
    s = sm.BatchSolver(N, 2 * N, B, n_plants=B)
    st = torch.cuda.Stream()
    Xbuf = torch.zeros(B * 4, dtype=torch.float64, device=dev)  # the same X/U pointers in every phase:
    Ud = torch.zeros(B, dtype=torch.float64, device=dev)        # only the generation tells the graphs apart
    for phase, nx in enumerate((4, 3, 4)):
        pl = dict(plant, Ad=plant["Ad"][:nx, :nx].copy(), Bd=plant["Bd"][:nx].copy(), Cd=plant["Cd"][:nx].copy(),
                  K=plant["K"][:nx].copy())
        Ad = np.tile(pl["Ad"], (B, 1, 1))
        Bd = np.tile(pl["Bd"], (B, 1))
        keep = [t(Ad), t(Bd), t(np.tile(pl["Cd"], (B, 1))), t(np.tile(pl["K"], (B, 1))), t(np.full(B, pl["Q"])),
                t(np.full(B, pl["R"])), t(np.full(B, pl["RD"]))]
        torch.cuda.synchronize()
        s.mpc_setup_plants_device(nx, 10, *[k.data_ptr() for k in keep], st.cuda_stream)
        st.synchronize()
        s.mpc_set_plant(Ad, Bd)
        X, U = workload.mpc_states(50 + phase, 0, B)
        X = X[:, :nx].copy()
        Xd = Xbuf[:B * nx]
        Xd.copy_(t(X.reshape(-1)))
        Ud.copy_(t(U))
        torch.cuda.synchronize()
        ops = oracle.condense(pl, N)
        l = np.full(2 * N, LMIN)
        refs = [oracle.Solver(ops["P"], np.zeros(N), ops["A"], l, ops["W0"]) for _ in range(B)]
        Xk, Uk = X.copy(), U.copy()
        for k in range(steps):
            with torch.cuda.stream(st):
                s.mpc_run_device(Xd.data_ptr(), Ud.data_ptr(), 0.0, 1, 9, 0, k, 1e-2, st.cuda_stream)
            st.synchronize()
            for b, r in enumerate(refs):
                assert r.update_gradient(oracle.gradient(ops, Xk[b], Uk[b]))
                assert r.update_upper_bound(oracle.upper_bound(ops, Xk[b], Uk[b]))
                if r.solve() == oracle.SOLVED:
                    Uk[b] += r.x()[0]
            np.testing.assert_allclose(Ud.cpu().numpy(), Uk, rtol=0, atol=1e-9, err_msg=f"phase {phase} step {k}")
            Xk = Xd.cpu().numpy().reshape(B, nx).copy()


def test_paired_tile_path_selected(plant):
    """The reference's constraint matrix Gbar = [K0 L; -K0 L] (ModelPredictiveControlAPI.cpp:332-347)
    puts a shared-plant batch on the tile kernel's paired loop; a generic A does not; batches under
    8,192 QPs run one QP per wave (the path mpcq_get_path reports is the one launch_args runs)."""
    N, B = 20, 8192
    ops, X, U, q, u = _problem(plant, N, B)
    s = _gpu_solve(ops, q, u, N, dtype="f32")
    assert s.path() == ("tile", True)
    A = ops["A"].copy()
    A[N + 3, 0] *= 1.0000001  # no longer an exact negation of row 3
    s2 = sm.BatchSolver(N, 2 * N, B, dtype="f32")
    s2.setup(ops["P"], np.zeros(N), A, np.full(2 * N, LMIN), ops["W0"])
    assert s2.path() == ("tile", False)
    s3 = _gpu_solve(ops, q[:64], u[:64], N, dtype="f32")
    assert s3.path() == ("wave", False)


class _DevArray:
    """A device buffer of the C ABI's device view, wrapped for torch (__cuda_array_interface__)."""

    def __init__(self, ptr, shape, typestr="<f8"):
        self.__cuda_array_interface__ = {"shape": shape, "typestr": typestr, "data": (ptr, False), "version": 3}


@pytest.mark.parametrize("dtype", ["f32", "f64"])
def test_tile_step_leaves_reference_qp_data(plant, dtype):
    """A tile-path controllerStep saves X and U; the solver's q and u (what updateGradient /
    updateUpperBound leave in OSQP, ModelPredictiveControlAPI.cpp:96-99) are computed from them when
    first read.  The device view must show the step's q, u bit-identical to an eager one-QP-per-wave
    step (same fp64 arithmetic), within 1e-12 of the oracle's; a generic solve after the step must
    solve that same QP (statuses and iterations of the step's solve, warm-started from its state)."""
    import torch

    N, B = 20, 8192
    ops, X, U, q, u = _problem(plant, N, B, seed=41)
    dev = torch.device("cuda:0")
    res = {}
    for kern in ("tile", "wave"):
        os.environ["MPCQ_KERNEL"] = kern
        try:
            s = sm.BatchSolver(N, 2 * N, B, dtype=dtype)
            s.setup(ops["P"], np.zeros(N), ops["A"], np.full(2 * N, LMIN), ops["W0"])
            s.mpc_set_operators(ops["Fx"], ops["Fu"], ops["Fr"], ops["Sbar"], ops["Ku"], ops["W0"])
            Xd = torch.from_numpy(X).to(dev)
            Ud = torch.from_numpy(U).to(dev)
            s.mpc_step_device(Xd.data_ptr(), Ud.data_ptr(), plant["xref"], torch.cuda.current_stream(dev).cuda_stream)
            assert s.path()[0] == kern
            v = s.device_view()
            torch.cuda.synchronize()
            qd = torch.as_tensor(_DevArray(v["q"], (B, N)), device=dev).cpu().numpy().copy()
            ud = torch.as_tensor(_DevArray(v["u"], (B, 2 * N)), device=dev).cpu().numpy().copy()
            res[kern] = (qd, ud, *s.info())
            if kern == "tile":  # a generic solve of the step's QP from the step's state
                st0, it0 = s.info()[:2]
                s.solve()
                st1, it1 = s.info()[:2]
                assert np.array_equal(st1, st0)
                assert np.all(it1 <= it0)  # (warm-started at the step's solution: at most as many)
            s.close()
        finally:
            os.environ.pop("MPCQ_KERNEL", None)
    assert np.array_equal(res["tile"][0], res["wave"][0]) and np.array_equal(res["tile"][1], res["wave"][1])
    assert np.abs(res["tile"][0] - q).max() <= 1e-12 * max(1.0, np.abs(q).max())
    assert np.abs(res["tile"][1] - u).max() <= 1e-12 * max(1.0, np.abs(u).max())


@pytest.mark.gpu
def test_phase_chain_counters_across_solves(plant, monkeypatch):
    """One context, consecutive cold solves whose phase chains differ in length (default, one launch,
    two launches, default again): the list counters the launches keep clean themselves (no per-solve
    memset) must hand every QP on, so each solve gives the first one's statuses, iterations and
    |dx| <= 1e-9 (f64), and the two default solves are bit-identical."""
    N, B = 20, 16384
    ops, X, U, q, u = _problem(plant, N, B, seed=29)
    s = _gpu_solve(ops, q, u, N, dtype="f64")
    x0, st0, it0, _ = (s.solution(), *s.info())
    assert np.all(st0 == sm.SOLVED)
    for phases in ("0", "3,5", None):
        if phases is None:
            monkeypatch.delenv("MPCQ_PHASES", raising=False)
        else:
            monkeypatch.setenv("MPCQ_PHASES", phases)
        s.reset_state()
        s.solve()
        x1, st1, it1, _ = (s.solution(), *s.info())
        assert np.array_equal(st1, st0), phases
        assert np.array_equal(it1, it0), phases
        assert np.abs(x1 - x0).max() <= 1e-9, phases
        if phases is None:
            assert np.array_equal(x1, x0)


def test_mimo_only_context_rejects_generic_calls(plant):
    """A per-plant context beyond the generic kernels' capacity (n = 40, m = 80) is MIMO-only: every
    generic entry point fails cleanly with MPCQ_ERR_ARG instead of touching its one-plant buffers."""
    from solvempc_amd import _capi
    N, B = 40, 16
    s = sm.BatchSolver(N, 2 * N, B, n_plants=B)
    ops = oracle.condense(plant, N)
    calls = [
        lambda: s.setup(np.tile(ops["P"], (B, 1, 1)), np.zeros((B, N)), np.tile(ops["A"], (B, 1, 1)),
                        np.full((B, 2 * N), LMIN), np.tile(ops["W0"], (B, 1))),
        lambda: s.mpc_set_operators(*[np.tile(ops[k], (B,) + (1,) * ops[k].ndim)
                                      for k in ("Fx", "Fu", "Fr", "Sbar", "Ku", "W0")]),
        lambda: s.mpc_set_plant(np.tile(plant["Ad"], (B, 1, 1)), np.tile(plant["Bd"], (B, 1))),
        lambda: s.mpc_setup_plants_device(4, 10, *([1] * 7)),
        lambda: s.solve(),
        lambda: s.warm_start(np.zeros((B, N)), np.zeros((B, 2 * N))),
        lambda: s.mpc_step(np.zeros((B, 4)), np.zeros(B)),
    ]
    for f in calls:
        with pytest.raises(sm.MpcqError) as e:
            f()
        assert e.value.code == _capi.MPCQ_ERR_ARG, e.value


def test_formulations_do_not_mix(plant):
    """mpcq_solve after a MIMO setup, and a MIMO step after a generic setup, fail with MPCQ_ERR_ORDER."""
    import torch
    from solvempc_amd import _capi
    N, B = 20, 8
    dev = torch.device("cuda:0")
    t = lambda a: torch.as_tensor(np.ascontiguousarray(a, dtype=np.float64), device=dev)  # noqa: E731
    s = sm.BatchSolver(N, 2 * N, B, n_plants=B)
    mimo = [t(np.tile(plant["Ad"], (B, 1, 1))), t(np.tile(plant["Bd"][:, None], (B, 1, 1))),
            t(np.tile(plant["Cd"][None], (B, 1, 1))), t(np.full((B, 1, 1), plant["Q"])), t(np.full((B, 1, 1), plant["R"])),
            t(np.full((B, 1, 1), plant["RD"])), t(np.tile(plant["K"][None], (B, 1, 1))),
            t(np.full((B, 1, 1), plant["K"][0])), t(np.full((B, 1), 255.0))]
    s.mimo_setup_plants_device(4, 1, 1, 10, *[x.data_ptr() for x in mimo])
    with pytest.raises(sm.MpcqError) as e:
        s.solve()
    assert e.value.code == _capi.MPCQ_ERR_ORDER
    siso = [t(np.tile(plant["Ad"], (B, 1, 1))), t(np.tile(plant["Bd"], (B, 1))), t(np.tile(plant["Cd"], (B, 1))),
            t(np.tile(plant["K"], (B, 1))), t(np.full(B, plant["Q"])), t(np.full(B, plant["R"])), t(np.full(B, plant["RD"]))]
    s.mpc_setup_plants_device(4, 10, *[x.data_ptr() for x in siso])
    Xd, Ud = t(np.zeros((B, 4))), t(np.zeros(B))
    with pytest.raises(sm.MpcqError) as e:
        s.mimo_step_device(Xd.data_ptr(), Ud.data_ptr())
    assert e.value.code == _capi.MPCQ_ERR_ORDER
    s.mpc_step_device(Xd.data_ptr(), Ud.data_ptr())  # the generic formulation runs
    torch.cuda.synchronize()
    assert np.all(s.info()[0] == sm.SOLVED)


@pytest.mark.parametrize("dtype", ["f32", "f64", "mixed"])
def test_results_independent_of_batch_order(plant, dtype, monkeypatch):
    """A QP's arithmetic does not depend on the wave or the other columns it runs with: the batch in
    index order and the same QPs in a random permutation give bit-identical solutions, duals,
    statuses and iteration counts on the tile path (generic solve and the controllerStep path)."""
    import torch
    N, B = 20, 16384
    ops, X, U, q, u = _problem(plant, N, B, seed=31)
    l = np.full(2 * N, LMIN)
    perm = np.random.default_rng(7).permutation(B)
    res = []
    for p in (np.arange(B), perm):
        s = _gpu_solve(ops, q[p], u[p], N, dtype=dtype)
        assert s.path()[0] == "tile"
        gen = (s.solution(), s.dual(), *s.info())
        m = sm.BatchSolver(N, 2 * N, B, dtype=dtype)
        m.setup(ops["P"], np.zeros(N), ops["A"], l, oracle.upper_bound(ops, np.zeros(4), 0.0))
        m.mpc_set_operators(ops["Fx"], ops["Fu"], ops["Fr"], ops["Sbar"], ops["Ku"], ops["W0"])
        Xd, Ud = torch.from_numpy(X[p].copy()).cuda(), torch.from_numpy(U[p].copy()).cuda()
        m.mpc_step_device(Xd.data_ptr(), Ud.data_ptr(), 0.0)
        torch.cuda.synchronize()
        inv = np.argsort(p)
        res.append([v[inv] for v in gen + (Ud.cpu().numpy(), m.solution(), *m.info())])
    assert np.all(res[0][2] == sm.SOLVED)
    for a, b in zip(res[0], res[1]):
        assert np.array_equal(a, b)


def test_verbose_stream_on_the_graph_path(plant, monkeypatch, capfd):
    """settings.verbose (setVerbosity, ModelPredictiveControlAPI.cpp:51) on mpcq_mpc_run_device's per-step
    graph path: the captured solve must not synchronise (that would invalidate the capture), so the summary
    is printed after each replayed step instead: one OSQP-style summary per control step, results bit-identical
    to the same stream without verbose."""
    import torch
    monkeypatch.setenv("MPCQ_STREAM", "graph")
    N, B, steps = 20, 64, 5
    ops = oracle.condense(plant, N)
    l = np.full(2 * N, LMIN)
    X, U = workload.stream_states(4, 0, B)

    def run(verbose):
        s = sm.BatchSolver(N, 2 * N, B, dtype="f64", settings=sm.default_settings(verbose=verbose))
        s.setup(ops["P"], np.zeros(N), ops["A"], l, oracle.upper_bound(ops, np.zeros(4), 0.0))
        s.mpc_set_operators(ops["Fx"], ops["Fu"], ops["Fr"], ops["Sbar"], ops["Ku"], ops["W0"])
        s.mpc_set_plant(plant["Ad"], plant["Bd"])
        Xd, Ud = torch.from_numpy(X.copy()).cuda(), torch.from_numpy(U.copy()).cuda()
        st = torch.cuda.Stream()
        with torch.cuda.stream(st):
            s.mpc_run_device(Xd.data_ptr(), Ud.data_ptr(), 0.0, steps, 4, 0, 0, 1e-2, st.cuda_stream)
        st.synchronize()
        assert s.stream_path() == "graph"
        return Xd.cpu().numpy(), Ud.cpu().numpy(), *s.info()

    quiet = run(0)
    capfd.readouterr()
    loud = run(1)
    out = capfd.readouterr().out
    for a_, b_ in zip(quiet, loud):
        assert np.array_equal(a_, b_)
    assert out.count("libmpcq: batched OSQP-v0.6 ADMM") == 1
    assert out.count("status:               solved") == steps, out[-2000:]
    assert out.count("number of iterations:") == steps


def _order_bin(v):
    """OrderBins::bin (mpcq_internal.h) on the host: 16 bins per octave of |v| (sub-octave steps linear in the
    fraction), 0 first, non-finite last."""
    a = np.abs(v)
    out = np.full(a.shape, 511, dtype=np.int64)
    fin = np.isfinite(a)
    f, e = np.frexp(a[fin])
    i = np.clip((e - 1) * 16 + ((f - 0.5) * 32.0).astype(np.int64) + 256, 0, 510)
    out[fin] = np.where(a[fin] == 0.0, 0, i)
    return out


@pytest.mark.parametrize("dtype", ["f64", "mixed"])
def test_ordered_step_ragged_batch_and_snapshot(plant, dtype, monkeypatch):
    """A ragged tile batch (10,001 QPs: a partial last wave, a partial last ordering workgroup) through the
    hardest-first step, and the step's q, u on demand from the order kernel's X, U snapshot (the ordered
    launch leaves the snapshot to mpcq_order.hip): every output and the device view's q, u bit-identical to
    index order (MPCQ_ORDER=0, whose tile launch takes the snapshot itself), q, u within 1e-12 of the
    oracle's (ModelPredictiveControlAPI.cpp:96-99)."""
    import torch
    N, B = 20, 10001
    ops, X, U, q, u = _problem(plant, N, B, seed=5)
    l = np.full(2 * N, LMIN)

    def run(order):
        if order:
            monkeypatch.delenv("MPCQ_ORDER", raising=False)
        else:
            monkeypatch.setenv("MPCQ_ORDER", "0")
        s = sm.BatchSolver(N, 2 * N, B, dtype=dtype)
        s.setup(ops["P"], np.zeros(N), ops["A"], l, oracle.upper_bound(ops, np.zeros(4), 0.0))
        s.mpc_set_operators(ops["Fx"], ops["Fu"], ops["Fr"], ops["Sbar"], ops["Ku"], ops["W0"])
        Xd, Ud = torch.from_numpy(X.copy()).cuda(), torch.from_numpy(U.copy()).cuda()
        s.mpc_step_device(Xd.data_ptr(), Ud.data_ptr(), 0.0)
        torch.cuda.synchronize()
        assert s.path()[0] == "tile"
        o = s.order()[0]
        v = s.device_view()
        torch.cuda.synchronize()
        qd = torch.as_tensor(_DevArray(v["q"], (B, N)), device="cuda").cpu().numpy()
        ud = torch.as_tensor(_DevArray(v["u"], (B, 2 * N)), device="cuda").cpu().numpy()
        out = (Ud.cpu().numpy(), s.solution(), s.dual(), *s.info(), qd, ud)
        s.close()
        return o, out

    o1, got = run(True)
    o0, ref = run(False)
    assert o1 and not o0
    for a_, b_ in zip(got, ref):
        assert np.array_equal(a_, b_, equal_nan=True)
    qd, ud = got[-2], got[-1]
    assert np.abs(qd - q).max() <= 1e-12 * max(1.0, np.abs(q).max())
    assert np.abs(ud - u).max() <= 1e-12 * max(1.0, np.abs(u).max())


@pytest.mark.parametrize("dtype", ["f64", "mixed"])
def test_ordered_step_lazy_info(plant, dtype, monkeypatch):
    """A hardest-first step in one launch stores (status, iter) in list-slot order, one 8-B store per QP
    into its wave's line (AdmmArgs::info_slot), and mpcq_api.cpp materialize_info permutes them when read:
    bit-identical to the stores at the QPs' indices (MPCQ_LAZY_INFO=0) whichever reader comes first
    (get_info; get_solution, whose publish kernel reads the status; the device view), and a step that
    nobody read is superseded by the next one (10,001 QPs: a ragged last wave)."""
    import torch
    N, B = 20, 10001
    ops, X, U, q, u = _problem(plant, N, B, seed=7)
    X2 = workload.mpc_states(8, 0, B, 1.0)[0]
    l = np.full(2 * N, LMIN)

    def run(lazy):
        if lazy:
            monkeypatch.delenv("MPCQ_LAZY_INFO", raising=False)
        else:
            monkeypatch.setenv("MPCQ_LAZY_INFO", "0")
        s = sm.BatchSolver(N, 2 * N, B, dtype=dtype)
        s.setup(ops["P"], np.zeros(N), ops["A"], l, oracle.upper_bound(ops, np.zeros(4), 0.0))
        s.mpc_set_operators(ops["Fx"], ops["Fu"], ops["Fr"], ops["Sbar"], ops["Ku"], ops["W0"])
        Xd, Ud = torch.from_numpy(X.copy()).cuda(), torch.from_numpy(U.copy()).cuda()
        out = []
        s.mpc_step_device(Xd.data_ptr(), Ud.data_ptr(), 0.0)  # step 1: info read first
        out += [*s.info(), s.solution()]
        s.mpc_step_device(Xd.data_ptr(), Ud.data_ptr(), 0.0)  # step 2: the solution read first
        out += [s.solution(), *s.info()]
        s.mpc_step_device(Xd.data_ptr(), Ud.data_ptr(), 0.0)  # step 3: nobody reads it
        Xd.copy_(torch.from_numpy(X2))
        s.mpc_step_device(Xd.data_ptr(), Ud.data_ptr(), 0.0)  # step 4: through the device view
        o = s.order()[0]
        v = s.device_view()
        torch.cuda.synchronize()
        out += [torch.as_tensor(_DevArray(v[k], (B,), "<i4"), device="cuda").cpu().numpy().copy()
                for k in ("status", "iter")]
        out += [Ud.cpu().numpy(), s.dual()]
        s.close()
        return o, out

    o1, got = run(True)
    o0, ref = run(False)
    assert o1 and o0  # both ran hardest-first; only the info stores differ
    for a_, b_ in zip(got, ref):
        assert np.array_equal(a_, b_, equal_nan=True)
    st4, it4 = got[-4], got[-3]
    assert (st4 == sm.SOLVED).mean() > 0.99 and it4.max() <= 4000


@pytest.mark.parametrize("dtype", ["f32", "f64", "mixed"])
def test_hardest_first_order_is_transparent(plant, dtype, monkeypatch):
    """The tile path's hardest-first MPC step (mpcq_order.hip: the batch run in ascending |max_j (A x_u -
    u)_j|, one launch) against the same step in index order with the phase chain (MPCQ_ORDER=0), on the
    bench's 65,536 QPs: every output bit-identical (U, x, y, status, iterations, rho), since a QP's
    arithmetic does not depend on its wave or launch.  The device's bins are the host's key binned the
    same way (the key from x_u = -P^-1 q on the oracle's q, u, up to rounding at bin edges), and the
    first bins hold the QPs that need the most iterations."""
    import torch
    N, B = 20, 65536
    ops, X, U, q, u = _problem(plant, N, B)
    l = np.full(2 * N, LMIN)

    def run(order):
        if order:
            monkeypatch.delenv("MPCQ_ORDER", raising=False)
        else:
            monkeypatch.setenv("MPCQ_ORDER", "0")
        s = sm.BatchSolver(N, 2 * N, B, dtype=dtype)
        s.setup(ops["P"], np.zeros(N), ops["A"], l, oracle.upper_bound(ops, np.zeros(4), 0.0))
        s.mpc_set_operators(ops["Fx"], ops["Fu"], ops["Fr"], ops["Sbar"], ops["Ku"], ops["W0"])
        Xd, Ud = torch.from_numpy(X.copy()).cuda(), torch.from_numpy(U.copy()).cuda()
        s.mpc_step_device(Xd.data_ptr(), Ud.data_ptr(), 0.0)
        torch.cuda.synchronize()
        o, order = s.order()
        out = (Ud.cpu().numpy(), s.solution(), s.dual(), *s.info())
        s.close()
        return o, order, out

    o1, order, got = run(True)
    o0, order0, ref = run(False)
    assert o1 and not o0 and np.array_equal(order0, np.arange(B))
    for a_, b_ in zip(got, ref):
        assert np.array_equal(a_, b_)
    assert np.array_equal(np.sort(order), np.arange(B))  # a permutation of the batch
    xu = -np.linalg.solve(ops["P"], q.T).T
    key = (xu @ ops["A"].T - u).max(axis=1)
    bins = _order_bin(key)[order]  # the host's bins along the device's order: ascending up to rounding at
    assert (np.diff(bins) < 0).sum() <= 2e-3 * B  # a bin edge (the device's key is the affine map's)
    # the first ~1 % of the order holds the slowest QPs: every QP needing more than 125 iterations
    it = ref[4]
    pos = np.empty(B, dtype=np.int64)
    pos[order] = np.arange(B)
    assert (pos[it > 125] < B // 100).all()


@pytest.mark.parametrize("dtype", ["f32", "f64", "mixed"])
def test_lazy_solution_publish_is_bit_identical(plant, dtype, monkeypatch):
    """A tile solve publishes x, y lazily (the finalize stores the warm state and U; mpcq_tile.h
    tile_publish_kernel forms x = D W x', y = E y / c when a caller reads them): bit-identical to the eager
    finalize (MPCQ_LAZY_XY=0) through get_solution / get_dual and the device view, NaN where OSQP publishes
    no solution (an infeasible QP among them), and still the last solve's after a cold start zeroes the warm
    state and after a reset (the next solve's fresh start)."""
    import torch
    N, B = 20, 16384
    ops, X, U, q, u = _problem(plant, N, B)
    u = u.copy()
    u[7:9, :N] = -1e3  # rows j and N + j: A_j x <= -1e3 and -A_j x <= -1e3 -> primal infeasible
    u[7:9, N:] = -1e3
    u[9, 3] = 1e30  # a row that would become free: TYPE_CHANGED (osqp_update_upper_bound's check), no solution

    def run(lazy):
        if lazy:
            monkeypatch.delenv("MPCQ_LAZY_XY", raising=False)
        else:
            monkeypatch.setenv("MPCQ_LAZY_XY", "0")
        s = _gpu_solve(ops, q, u, N, dtype=dtype)
        assert s.path()[0] == "tile"
        x, y = s.solution(), s.dual()
        v = s.device_view()
        torch.cuda.synchronize()
        xv = torch.as_tensor(_DevArray(v["x"], (B, N)), device="cuda").cpu().numpy()
        s.reset_state()
        x_r = s.solution()
        s.cold_start()
        x_c, y_c = s.solution(), s.dual()
        st = s.info()[0]
        s.close()
        return x, y, xv, x_r, x_c, y_c, st

    lz, eg = run(True), run(False)
    for a_, b_ in zip(lz, eg):
        assert np.array_equal(a_, b_, equal_nan=True)
    x, y, xv, x_r, x_c, y_c, st = lz
    no_sol = ~np.isin(st, (sm.SOLVED, sm.SOLVED_INACCURATE, sm.MAX_ITER_REACHED))
    assert no_sol[9] and st[9] == sm.TYPE_CHANGED
    # QPs 7, 8: OSQP's primal-infeasibility certificate (fp32: or MAX_ITER_REACHED, the bound documented at
    # test_infeasible_statuses_match_oracle)
    ok_inf = ((sm.PRIMAL_INFEASIBLE, sm.MAX_ITER_REACHED, sm.SOLVED_INACCURATE) if dtype == "f32"
              else (sm.PRIMAL_INFEASIBLE,))
    assert np.all(np.isin(st[7:9], ok_inf)), st[7:9]
    assert np.array_equal(np.isnan(x).all(axis=1), no_sol) and np.array_equal(np.isnan(y).all(axis=1), no_sol)
    assert np.array_equal(xv, x, equal_nan=True) and np.array_equal(x_r, x, equal_nan=True)
    assert np.array_equal(x_c, x, equal_nan=True) and np.array_equal(y_c, y, equal_nan=True)
