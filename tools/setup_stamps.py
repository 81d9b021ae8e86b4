"""Summarise MPCQ_MIMO_SETUP_STAMPS (dev tool): median cycles per setup phase."""
import sys

import numpy as np

r = np.fromfile(sys.argv[1], dtype=np.int64).reshape(-1, 16)
names = ["load", "recurrences", "Fx + QCS", "H + Fu/Frs", "symmetrize", "Ruiz x scaling", "outputs"]
for k, nm in enumerate(names):
    print(f"{nm:24s} {np.median(r[:, k + 1] - r[:, k]):10.0f}")
print(f"{'total':24s} {np.median(r[:, 7] - r[:, 0]):10.0f}")
if (r[:, 8] > 0).any():
    print("one Ruiz pass (pass 1):")
    for nm, a_, b_ in (("sweep wait", 8, 9), ("combine + mean + barrier", 9, 10), ("Dt/Et + barrier", 10, 11),
                       ("colpart + loop", 11, 8)):
        d = r[:, b_] - r[:, a_] if b_ > a_ else None
        if d is not None:
            print(f"  {nm:24s} {np.median(d):10.0f}")
