"""Summarise MPCQ_MIMO_SETUP_STAMPS (dev tool): median cycles per setup phase."""
import sys

import numpy as np

r = np.fromfile(sys.argv[1], dtype=np.int64).reshape(-1, 16)
names = ["load", "recurrences", "Fx + QCS", "H + Fu/Frs", "symmetrize", "Ruiz x scaling", "outputs"]
for k, nm in enumerate(names):
    print(f"{nm:24s} {np.median(r[:, k + 1] - r[:, k]):10.0f}")
print(f"{'total':24s} {np.median(r[:, 7] - r[:, 0]):10.0f}")
