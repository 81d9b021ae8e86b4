"""CPU tests of the checker itself (oracle/): pinned against the reference's known-answer values
(produced by a survey-time build of /root/reference's own
ModelPredictiveControlAPI.cpp) and certified by KKT conditions where no reference output exists."""
import numpy as np
import pytest

import oracle
from solvempc_amd import workload

LMIN = -np.finfo(np.float64).max


def test_condense_known_answers(plant):
    """SURVEY.md Appendix B KATs (N = 15, the reference's mpcWindow)."""
    o = oracle.condense(plant, 15)
    kat = {
        ("P", 0, 0): 11.000054467922261, ("P", 0, 1): 0.93338663476976957,
        ("P", 14, 14): 10.066666709654967, ("P", 0, 14): 0.066666845462466012,
        ("Fu", 0): 0.066721134682260722, ("Fu", 14): 0.066666845462466012,
        ("Su", 0, 0): -0.000112452562885, ("Su", 1, 0): -0.00035904021540417532,
    }
    for (name, *idx), v in kat.items():
        assert o[name][tuple(idx)] == pytest.approx(v, rel=1e-13, abs=1e-18), (name, idx)
    np.testing.assert_allclose(o["Fx"][0], [-0.048643271265083346, -0.0063463657998492186,
                                            0.01008331963724376, 0.0011545376299916823], rtol=1e-13)
    ev = np.linalg.eigvalsh(o["P"])
    assert ev[0] == pytest.approx(10.0168, abs=1e-4) and ev[-1] == pytest.approx(16.4972, abs=1e-4)
    L = np.tril(np.ones((15, 15)))
    np.testing.assert_array_equal(o["A"], np.vstack([-50 * L, 50 * L]))
    X = np.array([0.01, 0.0, 0.02, 0.0])
    u = oracle.upper_bound(o, X, 0.0)
    np.testing.assert_allclose(u, [364.5] * 10 + [255] * 5 + [145.5] * 10 + [255] * 5, rtol=1e-15)
    q = oracle.gradient(o, X, 0.0)
    assert q[0] == pytest.approx(-0.00028476631990595827, rel=1e-13)
    assert q[14] == pytest.approx(-1.5216160607417957e-06, rel=1e-12)
    o20 = oracle.condense(plant, 20)
    ev = np.linalg.eigvalsh(o20["P"])
    assert ev[0] == pytest.approx(10.0168, abs=1e-4) and ev[-1] == pytest.approx(21.3607, abs=1e-4)
    # S rows >= 10 are never written by the reference (:185) => zero; Sbar nonzero rows 0-9, 20-29
    nz = np.nonzero(np.abs(o20["Sbar"]).sum(axis=1))[0]
    np.testing.assert_array_equal(nz, list(range(10)) + list(range(20, 30)))


def test_quirks(plant):
    """Appendix A: Su strict upper triangle zero; Fu uses diag(LL' Rbar') = R (not LL' Rbar 1)."""
    o = oracle.condense(plant, 15)
    assert np.all(np.triu(o["Su"], 1) == 0)
    Q, R = plant["Q"], plant["R"]
    np.testing.assert_allclose(o["Fu"], 2 * (R + Q * o["Su"][:, 0] @ o["Su"]), rtol=1e-14)


@pytest.mark.parametrize("N", [15, 20])
def test_golden_regression(golden_dir, plant, N):
    """The oracle still reproduces the committed fixtures (tests/golden/make_golden.py)."""
    g = np.load(golden_dir / f"qp_n{N}.npz", allow_pickle=False)
    o = oracle.condense(plant, N)
    for k in ("P", "A", "Fx", "Fu", "Fr", "Sbar", "Ku", "W0"):
        np.testing.assert_allclose(o[k], g[k], rtol=1e-15, atol=0, err_msg=k)
    np.testing.assert_allclose(oracle.gradient(o, g["X"], g["U"]), g["q"], rtol=1e-14, atol=1e-300)
    x, st, it, rho = oracle.batch_solve(o["P"], o["A"], np.zeros(N), np.full(2 * N, LMIN),
                                        oracle.upper_bound(o, np.zeros(4), 0.0), g["q"], g["u"], nthreads=1)
    np.testing.assert_array_equal(st, g["status"])
    np.testing.assert_array_equal(it, g["iter"])
    np.testing.assert_allclose(x, g["x"], rtol=0, atol=1e-12)


@pytest.mark.parametrize("N", [15, 20])
def test_tight_solution_is_kkt_optimal(golden_dir, plant, N):
    """Optimum mode: at eps 1e-10 the restatement satisfies KKT (independent of OSQP)."""
    g = np.load(golden_dir / f"qp_n{N}.npz", allow_pickle=False)
    o = oracle.condense(plant, N)
    l = np.full(2 * N, LMIN)
    s = oracle.Solver(o["P"], np.zeros(N), o["A"], l, oracle.upper_bound(o, np.zeros(4), 0.0),
                      oracle.default_settings(eps_abs=1e-10, eps_rel=1e-10, max_iter=200000))
    for b in range(0, 64, 8):
        assert s.update_gradient(g["q"][b]) and s.update_upper_bound(g["u"][b])
        assert s.solve() == oracle.SOLVED
        r = oracle.kkt_residuals(o["P"], g["q"][b], o["A"], l, g["u"][b], s.x(), s.y())
        scale = 1 + np.abs(g["q"][b]).max() + np.abs(o["A"].T @ s.y()).max()
        assert r["stationarity"] < 1e-7 * scale and r["primal"] < 1e-7 * (1 + np.abs(g["u"][b]).max())
        assert r["dual_sign"] < 1e-12 * scale and r["complementarity"] < 1e-5 * scale
        np.testing.assert_allclose(s.x(), g["x_opt"][b], atol=1e-6)
    # default-eps answers are close to, but not at, the optimum
    assert np.abs(g["x"] - g["x_opt"]).max() < 0.2


def test_osqp_scaling_and_defaults(plant):
    o = oracle.condense(plant, 20)
    s = oracle.Solver(o["P"], np.zeros(20), o["A"], np.full(40, LMIN), oracle.upper_bound(o, np.zeros(4), 0.0))
    D, E, c = s.scaling()
    np.testing.assert_allclose(D, 1 / np.sqrt(50), rtol=1e-14)  # A entries +-50 dominate Ruiz
    np.testing.assert_allclose(E, 1 / np.sqrt(50), rtol=1e-14)
    assert c == 1.0  # q == 0 at setup => cost scaling limited to 1 (scaling.c)
    st = oracle.default_settings()
    assert (st.rho, st.sigma, st.alpha, st.max_iter, st.check_termination, st.scaling) == (0.1, 1e-6, 1.6, 4000, 25, 10)


def test_infeasibility_statuses():
    P = np.eye(2)
    A = np.array([[1.0, 0.0], [1.0, 0.0]])
    s = oracle.Solver(P, np.zeros(2), A, np.array([-1e30, 1.0]), np.array([-1.0, 1e30]))
    assert s.solve() == oracle.PRIMAL_INFEASIBLE
    assert np.all(np.isnan(s.x()))
    # dual infeasible: P = 0 (PSD), q = (-1, 0), x0 unbounded above
    s = oracle.Solver(np.zeros((2, 2)), np.array([-1.0, 0.0]), np.array([[0.0, 1.0]]), np.array([-1.0]), np.array([1.0]))
    assert s.solve() == oracle.DUAL_INFEASIBLE


def test_max_iter_and_warm_start(plant):
    o = oracle.condense(plant, 20)
    X, U = workload.mpc_states(1, 0, 1)
    q, u = oracle.gradient(o, X, U)[0], oracle.upper_bound(o, X, U)[0]
    l = np.full(40, LMIN)
    s = oracle.Solver(o["P"], np.zeros(20), o["A"], l, oracle.upper_bound(o, np.zeros(4), 0.0),
                      oracle.default_settings(max_iter=10, eps_abs=1e-12, eps_rel=1e-12))
    s.update_gradient(q)
    s.update_upper_bound(u)
    assert s.solve() == oracle.MAX_ITER_REACHED and s.info().iter == 10
    # warm start: a second solve of the same data converges in one check interval
    s2 = oracle.Solver(o["P"], np.zeros(20), o["A"], l, oracle.upper_bound(o, np.zeros(4), 0.0))
    s2.update_gradient(q)
    s2.update_upper_bound(u)
    assert s2.solve() == oracle.SOLVED
    s2.update_gradient(q)
    s2.update_upper_bound(u)
    assert s2.solve() == oracle.SOLVED and s2.info().iter == 25


def test_plants_step_matches_per_plant_solver(plant):
    """oracle.plants_step (config-3 CPU path / baseline) == condense + Solver per plant; the
    randomised plants are shard-invariant and stable."""
    from solvempc_amd import workload

    B, N = 24, 20
    Ad, Bd = workload.randomized_plants(plant, 2, 100, B)
    A2, B2 = workload.randomized_plants(plant, 2, 110, 4)
    assert np.array_equal(A2, Ad[10:14]) and np.array_equal(B2, Bd[10:14])
    assert np.abs(np.linalg.eigvals(Ad)).max() < 1.0
    X, U = workload.mpc_states(3, 0, B)
    Uo, st, it = oracle.plants_step(plant, Ad, Bd, X, U, N, nthreads=2)
    for b in range(B):
        ops = oracle.condense(dict(plant, Ad=Ad[b], Bd=Bd[b]), N)
        r = oracle.Solver(ops["P"], np.zeros(N), ops["A"], np.full(2 * N, -np.finfo(np.float64).max),
                          oracle.upper_bound(ops, np.zeros(4), 0.0))
        assert r.update_gradient(oracle.gradient(ops, X[b], U[b]))
        assert r.update_upper_bound(oracle.upper_bound(ops, X[b], U[b]))
        s = r.solve()
        assert st[b] == s and it[b] == r.info().iter
        # (numpy's q/u products round differently from the C loops in the last bits)
        assert abs(Uo[b] - (U[b] + r.x()[0] if s == 1 else U[b])) < 1e-12


def test_mimo_condensing_siso_specialisation_is_bit_identical(plant):
    """oracle/mpc_mimo.c at n_u = n_y = 1, K0 = K(0), w0 = 255 reproduces the reference-pinned SISO
    condensing (mpc_condense.c, ModelPredictiveControlAPI.cpp:180-369) bit for bit."""
    for N in (15, 20):
        ref = oracle.condense(plant, N)
        mp = {"Ad": plant["Ad"], "Bd": plant["Bd"][:, None], "Cd": plant["Cd"][None, :], "Q": [[plant["Q"]]],
              "R": [[plant["R"]]], "RD": [[plant["RD"]]], "K": plant["K"][None, :], "K0": [[plant["K"][0]]],
              "w0": [255.0]}
        mo = oracle.condense_mimo(mp, N, s_rows=10)
        for k in ("P", "A", "Fx", "Fr", "Sbar", "W0", "Su"):
            assert np.array_equal(mo[k].reshape(ref[k].shape), ref[k]), (N, k)
        assert np.array_equal(mo["Fu"][:, 0], ref["Fu"]) and np.array_equal(mo["Ku"][:, 0], ref["Ku"])


def test_quadrotor_plants_and_oracle_solve():
    """Config 4 plants: exact ZOH of the hover model (the augmented matrix is nilpotent), mass/inertia
    spread within +-10%, and the oracle solves every sampled QP."""
    from solvempc_amd import workload

    Ad, Bd = workload.quadrotor_plants(3, 0, 8)
    A, B = workload.quadrotor_continuous(0.5, 2.3e-3, 2.3e-3, 4e-3)
    Ad0, Bd0 = workload.zoh(A, B, 0.02)
    assert np.allclose(Ad0, Ad[0])  # Ad does not depend on mass / inertia
    f = workload.QUAD["mass"] / (1.0 / Bd[:, 8, 0] * 0.02)  # Bd[8, 0] = dt / m
    assert np.all(np.abs(f - 1.0) <= 0.1 + 1e-12)
    X, U = workload.quadrotor_states(3, 0, 8)
    Un, x, st, it = oracle.mimo_plants_step(workload.quadrotor_shared(), Ad, Bd, X, U, 30, nthreads=4)
    assert np.all(st == oracle.SOLVED)
    assert np.all(np.abs(Un) <= np.array(workload.QUAD["w0"]) + 1e-3)  # the applied input stays in the box


def test_stream_workload_closed_loop_is_bounded():
    """Config 5's initial-state law (workload.stream_states) keeps the reference controller's closed
    loop (oracle controllerStep + X <- Ad X + Bd U + w, noise std 1e-2) SOLVED and bounded, where the
    config-2 law saturates the inner loop and diverges (workload.STREAM_X_SCALE)."""
    from solvempc_amd import workload

    plant = workload.reference_plant()
    N, B, steps = 20, 8, 300
    ops = oracle.condense(plant, N)
    l = np.full(2 * N, -np.finfo(np.float64).max)
    for law, bounded in (("stream", True), ("cfg2", False)):
        X, U = workload.stream_states(4, 0, B) if law == "stream" else workload.mpc_states(4, 0, B)
        rs = [oracle.Solver(ops["P"], np.zeros(N), ops["A"], l, ops["W0"]) for _ in range(B)]
        for k in range(steps):
            for b, r in enumerate(rs):
                assert r.update_gradient(oracle.gradient(ops, X[b], U[b]))
                assert r.update_upper_bound(oracle.upper_bound(ops, X[b], U[b]))
                if r.solve() == oracle.SOLVED:
                    U[b] += r.x()[0]
                else:
                    assert not bounded
            X = workload.simulate(plant["Ad"], plant["Bd"], X, U, workload.plant_noise(4, 0, B, k, 4, 1e-2))
        assert (np.abs(X).max() < 10) == bounded, (law, np.abs(X).max())


def test_stream_run_matches_python_replay(plant):
    """oracle.stream_run (the config-5 CPU baseline: one warm-started solver per plant, the device's
    noise stream) against a step-by-step replay with oracle.Solver and workload.simulate."""
    N, B, steps = 20, 5, 10
    X, U = workload.stream_states(4, 0, B)
    Xc, Uc, it, un = oracle.stream_run(plant, X, U, N, steps, 4, 0, 0, 1e-2)
    ops = oracle.condense(plant, N)
    l = np.full(2 * N, -np.finfo(np.float64).max)
    refs = [oracle.Solver(ops["P"], np.zeros(N), ops["A"], l, oracle.upper_bound(ops, np.zeros(4), 0.0))
            for _ in range(B)]
    Xk, Uk, its = X.copy(), U.copy(), np.zeros(B, dtype=np.int64)
    for k in range(steps):
        for b, r in enumerate(refs):
            assert r.update_gradient(oracle.gradient(ops, Xk[b], Uk[b]))
            assert r.update_upper_bound(oracle.upper_bound(ops, Xk[b], Uk[b]))
            if r.solve() == oracle.SOLVED:
                Uk[b] += r.x()[0]
            its[b] += r.info().iter
        Xk = workload.simulate(plant["Ad"], plant["Bd"], Xk, Uk, workload.plant_noise(4, 0, B, k, 4, 1e-2))
    assert np.array_equal(it, its) and np.all(un == 0)
    np.testing.assert_allclose(Uc, Uk, rtol=0, atol=1e-12)
    np.testing.assert_allclose(Xc, Xk, rtol=0, atol=1e-12)


def test_stream_run_rejects_shapes_beyond_its_buffers(plant):
    """ora_stream_run keeps q, u, x_next per thread in fixed buffers (N <= 64, nx <= 8): larger shapes are
    rejected, not written past the end."""
    import pytest

    X, U = np.zeros((2, 4)), np.zeros(2)
    with pytest.raises(ValueError):
        oracle.stream_run(plant, X, U, 65, 1, 4)
    with pytest.raises(ValueError):
        oracle.stream_run(plant, np.zeros((2, 9)), U, 20, 1, 4)
