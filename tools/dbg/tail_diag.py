# dev diagnostic: cfg2 batch, wave-kernel tail vs tile tail against the oracle on the long-tail QPs
import os, sys, numpy as np, torch
sys.path.insert(0, os.getcwd())
import solvempc_amd as sm, oracle
from solvempc_amd import workload
from tests.test_gpu import _problem, LMIN
plant = workload.reference_plant()
N, B = 20, 65536
ops, X, U, q, u = _problem(plant, N, B)
res = {}
for tail in ("wave", "tile"):
    os.environ["MPCQ_TAIL"] = tail
    for dt in ("f32", "f64"):
        s = sm.BatchSolver(N, 2 * N, B, dtype=dt)
        s.setup(ops["P"], np.zeros(N), ops["A"], np.full(2 * N, LMIN), oracle.upper_bound(ops, np.zeros(4), 0.0))
        s.update_lin_cost(q); s.update_upper_bound(u); s.solve()
        res[(tail, dt)] = (s.solution(), *s.info())
idx = np.nonzero((res[("tile", "f32")][2] > 125) | (res[("wave", "f32")][2] > 125))[0]
x_ref, st_ref, it_ref, _, margin = oracle.batch_solve(ops["P"], ops["A"], np.zeros(N), np.full(2 * N, LMIN),
    oracle.upper_bound(ops, np.zeros(4), 0.0), q[idx], u[idx], margins=True)
print("tail QPs", len(idx))
for k, (x, st, it, rho) in res.items():
    d = it[idx] != it_ref
    print(k, "it mismatches", int(d.sum()), "non-tie", int((d & (margin >= 2e-3)).sum()),
          "max|dx|", float(np.abs(x[idx] - x_ref).max()))
    for j in np.nonzero(d)[0][:6]:
        print("   qp", idx[j], "it", it[idx[j]], "ref", it_ref[j], "margin", margin[j], "rho", rho[idx[j]])
