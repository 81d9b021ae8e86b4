"""Summarise MPCQ_TILE_STAMPS output (dev tool): per phase launch, per-wave stage durations in shader
cycles (median / p90 / max over the waves that ran) and the launch span from s_memrealtime (100 MHz)."""
import sys

import numpy as np

f = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/stamps.bin"
raw = np.fromfile(f, dtype=np.int64)
nph, waves = int(raw[0]), int(raw[1])
st = raw[2:].reshape(nph, waves, 8)
for p in range(nph):
    s = st[p]
    ran = s[:, 0] != 0
    s = s[ran]
    if not len(s):
        print(f"phase {p}: no waves")
        continue
    looped = s[:, 2] != 0
    def q(v):
        v = v[v > 0] if (v > 0).any() else v
        return f"med {np.median(v):8.0f} p90 {np.percentile(v, 90):8.0f} max {v.max():8.0f}"
    img = s[:, 1] - s[:, 0]
    pro = np.where(looped, s[:, 2] - s[:, 1], 0)
    end = np.where(s[:, 3] != 0, s[:, 3], s[:, 4])
    loop = np.where(looped, end - s[:, 2], 0)
    save = np.where(s[:, 3] != 0, s[:, 4] - s[:, 3], 0)
    rt0, rt1 = s[:, 6], s[:, 7]
    span = (rt1.max() - rt0.min()) / 100.0  # us
    skew = (np.percentile(rt0, 99) - rt0.min()) / 100.0
    print(f"phase {p}: waves {len(s)} looped {looped.sum()}  span {span:.1f} us  entry skew(p99) {skew:.1f} us")
    info = np.where(looped, s[:, 5], 0)  # non-zero only in a -DMPCQ_INFO_STAMPS build
    print(f"   image+barrier {q(img)}\n   prologue      {q(pro)}\n   loop          {q(loop)}\n"
          f"    of which info iterations {q(info)}\n   save          {q(save)}")
    lat = (rt1 - rt0) / 100.0
    print(f"   wave lifetime us: med {np.median(lat):.1f} max {lat.max():.1f}; exits in last 10% of span: "
          f"{np.mean(rt1 > rt0.min() + 0.9 * span * 100):.2%}")
