"""Summarise MPCQ_TILE_STAMPS of a work-queue solve (dev tool): per wave the groups and QPs it ran,
the cycles inside groups vs its lifetime, and the exit-time distribution (s_memrealtime, 100 MHz)."""
import sys

import numpy as np

raw = np.fromfile(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/stamps.bin", dtype=np.int64)
nph, waves = int(raw[0]), int(raw[1])
s = raw[2:2 + waves * 8].reshape(waves, 8)
s = s[s[:, 0] != 0]
groups, qps, busy = s[:, 2], s[:, 3], s[:, 5]
life = s[:, 4] - s[:, 1]
rt0, rt1 = s[:, 6], s[:, 7]
span = (rt1.max() - rt0.min()) / 100.0
print(f"waves {len(s)}  span {span:.1f} us  groups {groups.sum()} (per wave med {np.median(groups):.0f} max {groups.max()})  "
      f"QPs {qps.sum()}  mean QPs/group {qps.sum() / max(1, groups.sum()):.2f}")
print(f"busy/lifetime: med {np.median(busy / np.maximum(life, 1)):.3f}  total busy cycles {busy.sum():.3e}  "
      f"image+barrier med {np.median(s[:, 1] - s[:, 0]):.0f} cycles")
ex = (rt1 - rt0.min()) / 100.0
print("exit time us percentiles 10/50/90/99/100:", np.percentile(ex, [10, 50, 90, 99, 100]).round(1))
print("entry time us p99:", np.percentile((rt0 - rt0.min()) / 100.0, 99).round(1))
