"""Regenerate the golden fixtures in tests/golden/ from the CPU oracle (oracle/).

The reference (LukeSchmitt96/solveMPC) ships no tests or fixtures and is unbuildable here (its QP code
needs OsqpEigen and Eigen's unsupported/MatrixFunctions, both absent), so these vectors come from the
oracle's restatement, whose condensing is pinned by the known-answer values in SURVEY.md Appendix B
(tests/test_oracle.py::test_condense_known_answers).  Run:  python tests/golden/make_golden.py
"""
from pathlib import Path
import sys

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

import oracle  # noqa: E402
from solvempc_amd import workload  # noqa: E402

OUT = Path(__file__).resolve().parent


def main():
    plant = workload.reference_plant()
    for N, u_range in ((15, 0.0), (20, 1.0)):
        ops = oracle.condense(plant, N)
        B = 64
        X, U = workload.mpc_states(1, 0, B, u_range)
        q = oracle.gradient(ops, X, U)
        u = oracle.upper_bound(ops, X, U)
        l = np.full(2 * N, -np.finfo(np.float64).max)
        q0, u0 = np.zeros(N), oracle.upper_bound(ops, np.zeros(4), 0.0)
        x, st, it, rho = oracle.batch_solve(ops["P"], ops["A"], q0, l, u0, q, u)
        tight = oracle.default_settings(eps_abs=1e-10, eps_rel=1e-10, max_iter=200000)
        xt, stt, itt, _ = oracle.batch_solve(ops["P"], ops["A"], q0, l, u0, q, u, settings=tight)
        np.savez_compressed(
            OUT / f"qp_n{N}.npz",
            **{k: v for k, v in ops.items()},
            X=X, U=U, q=q, u=u, x=x, status=st, iter=it, rho=rho, x_opt=xt, status_opt=stt,
        )
        print(f"qp_n{N}.npz: iters {np.unique(it, return_counts=True)}")


if __name__ == "__main__":
    main()
