"""Summarise the MPCQ_GJ_STAMPS debug build's stamps (dev tool): python tools/gj_stamps.py file"""
import sys

import numpy as np

r = np.fromfile(sys.argv[1], dtype=np.int64).reshape(-1, 8)
A, C, Cend, A80, C80, A41 = r[:, 2], r[:, 3], r[:, 4], r[:, 5], r[:, 6], r[:, 7]
ok = (A > 0) & (A41 > 0)
r = r[ok]
A, C, Cend, A80, C80, A41 = A[ok], C[ok], Cend[ok], A80[ok], C80[ok], A41[ok]
med = lambda v: float(np.median(v))  # noqa: E731
print(f"QPs {ok.sum()}: step 40 -> 41 barrier-to-barrier {med(A41 - A):.0f} cycles")
print(f"  t0 : after barrier -> FMAs done {med(C - A):.0f}; -> step end {med(Cend - A):.0f}")
print(f"  t80 (row owner of 41): barrier skew vs t0 {med(A80 - A):.0f}; after barrier -> its step end {med(C80 - A80):.0f}")
print(f"  t80 step end -> next barrier release (t0) {med(A41 - C80):.0f}")
