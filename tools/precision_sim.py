"""Diagnostic (CPU): where the fp32 tile path's distance from the fp64 trajectory comes from, and
what a mixed-precision schedule buys.

A numpy restatement of the tile kernel's W-basis paired ADMM (mpcq_tile.h) on a batch
of config-2 QPs (checks in fp64 from the state), each iteration in fp32 (state, plant data and the
three products rounded to fp32, fp32 accumulation) or fp64, compared with the all-fp64 run:

  python tools/precision_sim.py [B]

Modes:
  f32           every iteration in fp32 (the f32 tile path)
  state64       fp64 state, fp32 products (the products' fp32 accumulation remains)
  tail R        the last R iterations of every check interval in fp64, the rest in fp32 (the
                mixed tile path: checks, adapt_rho and the solution come from an fp64 state whose
                fp32 error the R fp64 iterations have damped)
"""
import os
import sys

import numpy as np
import scipy.linalg as sla

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle  # noqa: E402
from solvempc_amd import workload  # noqa: E402

N = 20
B = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
plant = workload.reference_plant()
ops = oracle.condense(plant, N)
P, A = ops["P"], ops["A"]
n, m = N, 2 * N
l = np.full(m, -np.finfo(np.float64).max)
u0 = oracle.upper_bound(ops, np.zeros(4), 0.0)
D, E, c = oracle.Solver(P, np.zeros(n), A, l, u0).scaling()
Ph = c * (D[:, None] * P * D[None, :])
Ah = E[:, None] * A * D[None, :]
sigma, alpha, rho0 = 1e-6, 1.6, 0.1
lam, W = sla.eigh(Ah.T @ Ah, Ph + sigma * np.eye(n))  # W'(P^+sI)W = I, W'A^'A^W = diag(lam)
Bt = (Ah @ W)[:n]  # top half of B = A^W; B_{n+j} = -B_j
S = sigma * W.T @ W

X, U = workload.mpc_states(1, 0, B)
qh = c * D[None, :] * oracle.gradient(ops, X, U)
uh = E[None, :] * oracle.upper_bound(ops, X, U)


def f32(a):
    return a.astype(np.float32).astype(np.float64)


def mm32(Mt, v):
    return (v.astype(np.float32) @ Mt.astype(np.float32)).astype(np.float64)


def mm64(Mt, v):
    return v @ Mt


def run(mode: str, R: int = 0):
    """mode: 'f64', 'f32', 'state64' or 'tail' (last R iterations of each interval in fp64)."""
    g64, g32 = -(qh @ W), f32(-mm32(W, qh))
    xs, z, y = np.zeros((B, n)), np.zeros((B, m)), np.zeros((B, m))
    rho = np.full(B, rho0)
    done, iters, xout = np.zeros(B, bool), np.zeros(B, int), np.zeros((B, n))
    for it in range(1, 4001):
        if mode == "f64" or (mode == "tail" and (it - 1) % 25 >= 25 - R):
            rr, mm, gg, ub = (lambda v: v), mm64, g64, uh
        elif mode == "state64":
            rr, mm, gg, ub = (lambda v: v), mm32, g32, f32(uh)
        else:
            rr, mm, gg, ub = f32, mm32, g32, f32(uh)
            xs, z, y = f32(xs), f32(z), f32(y)
        w = rho[:, None] * z - y
        wt = rr(w[:, :n] - w[:, n:])
        xi = rr(rr(gg + mm(S, xs)) + mm(Bt, wt))
        eta = rr(xi / (1.0 + rho[:, None] * lam[None, :]))
        xs = rr(alpha * eta + (1 - alpha) * xs)
        ztt = mm(Bt.T, eta)
        v = rr(alpha * np.concatenate([ztt, -ztt], axis=1) + (1 - alpha) * z)
        zn = np.minimum(rr(v + y / rho[:, None]), ub)
        y = rr(y + rho[:, None] * (v - zn))
        z = zn
        if it % 25 == 0:  # check_termination (unscaled), adapt_rho every 100 (OSQP v0.6)
            xh = xs @ W.T
            ax, px, aty = xh @ Ah.T, xh @ Ph.T, y @ Ah
            Ei, Di = 1 / E, 1 / D
            pri = np.abs(Ei * (ax - z)).max(1)
            epri = 1e-3 + 1e-3 * np.maximum(np.abs(Ei * ax).max(1), np.abs(Ei * z).max(1))
            dua = np.abs(Di * (px + qh + aty)).max(1) / c
            edua = 1e-3 + 1e-3 / c * np.maximum(np.maximum(np.abs(Di * px).max(1), np.abs(Di * aty).max(1)),
                                                np.abs(Di * qh).max(1))
            term = (~done) & (pri < epri) & (dua < edua)
            xout[term] = (xh * D)[term]
            iters[term] = it
            done |= term
            if it % 100 == 0:
                prn = np.abs(ax - z).max(1) / (np.maximum(np.abs(z).max(1), np.abs(ax).max(1)) + 1e-30)
                dun = np.abs(px + qh + aty).max(1) / (
                    np.maximum(np.maximum(np.abs(qh).max(1), np.abs(aty).max(1)), np.abs(px).max(1)) + 1e-30)
                rn = np.clip(rho * np.sqrt(prn / (dun + 1e-30)), 1e-6, 1e6)
                rho = np.where((~done) & ((rn > 5 * rho) | (rn < rho / 5)), rn, rho)
            if done.all():
                break
    return xout, iters


if __name__ == "__main__":
    ref, iref = run("f64")
    print(f"B={B}; fp64 iterations mean {iref.mean():.2f} max {iref.max()}; |x0| max {np.abs(ref[:, 0]).max():.2f}")
    for mode, R in [("f32", 0), ("state64", 0)] + [("tail", r) for r in (4, 6, 8, 10)]:
        x, its = run(mode, R)
        same = its == iref
        d0 = np.abs(x[:, 0] - ref[:, 0])
        print(f"{mode:8s} R={R:2d}: schedule differs {(~same).sum():4d}  max|dx0| {d0[same].max():.2e}  "
              f"max|dx| {np.abs(x - ref)[same].max():.2e}  fp64 share of iterations {R / 25:.2f}", flush=True)
