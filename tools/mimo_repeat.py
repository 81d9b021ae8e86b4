"""Dev tool: repeat the general-K0 MIMO parity case (tests/test_mimo.py) a few times on one library and
print the max relative x error against the oracle per run (determinism check)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
os.environ.setdefault("MPCQ_MIMO_GENERAL_K0", "1")
import oracle  # noqa: E402
from solvempc_amd import workload  # noqa: E402
import test_mimo as tm  # noqa: E402

N, B = 30, 12
Ad, Bd = workload.quadrotor_plants(9, 0, B)
sh = workload.quadrotor_shared()
X, U = workload.quadrotor_states(9, 0, B)
U_ref, x_ref, st_ref, it_ref, mg = oracle.mimo_plants_step(sh, Ad, Bd, X, U, N, nthreads=8, margins=True)
_orig = tm.sm.BatchSolver.info


def _info(self):
    st, it, rho = _orig(self)
    print("rho", np.array2string(rho, precision=6), flush=True)
    return st, it, rho


tm.sm.BatchSolver.info = _info
for r in range(int(sys.argv[1]) if len(sys.argv) > 1 else 4):
    Us, x, st, it = tm._run_device(sh, Ad, Bd, X, U, N)
    rel = np.abs(x - x_ref).max(axis=1) / np.maximum(1.0, np.abs(x_ref).max(axis=1))
    print(r, "status ok" if np.array_equal(st, st_ref) else "status DIFF", "iters", (it == it_ref).all(),
          "rel per QP", np.array2string(rel, precision=1), flush=True)
