"""Per-QP stage stamps of mimo_solve_kernel (dev tool; a debug build with MPCQ_DEBUG_HOOKS and
MPCQ_MIMO_STAMPS=file): slots 0 start, 1 front end done, 2 after the last factorisation, 3 end,
4 iterations, 5 factorisations.  Prints the stage means and a least-squares split of the solve
time into cycles per iteration and per factorisation."""
import sys

import numpy as np

s = np.fromfile(sys.argv[1], dtype=np.int64).reshape(-1, 8)
s = s[s[:, 3] > 0]
front = s[:, 1] - s[:, 0]
solve = s[:, 3] - s[:, 1]
it, nf = s[:, 4].astype(float), s[:, 5].astype(float)
one = nf == 1
print(f"QPs {len(s)}  front end {front.mean():.0f}  solve {solve.mean():.0f} cycles (mean)")
print(f"iterations mean {it.mean():.1f}  factorisations mean {nf.mean():.3f}")
fact1 = (s[one, 2] - s[one, 1])
print(f"first factorisation (QPs with one): {fact1.mean():.0f} cycles")
X = np.stack([it, nf, np.ones_like(it)], 1)
coef, *_ = np.linalg.lstsq(X, solve.astype(float), rcond=None)
print(f"solve ~ {coef[0]:.0f} x iterations + {coef[1]:.0f} x factorisations + {coef[2]:.0f}")
print(f"share: iterations {coef[0] * it.mean() / solve.mean():.3f}  factorisations {coef[1] * nf.mean() / solve.mean():.3f}")
