"""Summarise the MPCQ_WAVE_STAMPS debug build (dev tool): one plain tail iteration (140) of the
one-QP-per-wave kernel, stage by stage, from the MPCQ_TILE_STAMPS dump's last (wave) phase."""
import sys

import numpy as np

raw = np.fromfile(sys.argv[1], dtype=np.int64)
nph, waves = int(raw[0]), int(raw[1])
st = raw[2:].reshape(nph, waves * 8)[nph - 1][: 2048 * 16].reshape(2048, 16)
ok = (st[:, 0] > 0) & (st[:, 8] > 0) & (st[:, 4] > 0)
s = st[ok]
print(f"QPs sampled {ok.sum()}")
names = ["w, write x', w; barrier", "x-side products (S x' + B' w)", "eta write; barrier", "z-side product + projection"]
for k, nm in enumerate(names):
    print(f"  {nm:34s} {np.median(s[:, k + 1] - s[:, k]):8.0f}")
print(f"  {'whole iteration (140 -> 141)':34s} {np.median(s[:, 8] - s[:, 0]):8.0f}")
