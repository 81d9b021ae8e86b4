"""Per-plant stage stamps of mimo_setup_kernel (dev tool; a debug build, `SRC=mpcq_mimo.hip bash
tools/build_dbg.sh` -> tools/dbglib/libmpcq.so, run with MPCQ_LIBRARY pointing at it).  Runs the config-4
setup twice (the second timed) and prints the median shader cycles of each stage: 0 entry, 1 plant data in
LDS, 2 transformations (powers, CS), 3 Fx (MFMA) + QCS, 4 setH (MFMA) + Fu scan + Frs, 5 symmetrise,
6 Ruiz done, 7 outputs written.  Usage: python tools/mimo_setup_stamps.py [plants]"""
import os
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import solvempc_amd as sm  # noqa: E402
from solvempc_amd import workload  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
N, nu = 30, 4
out = os.environ.get("MPCQ_MIMO_SETUP_STAMPS", "/tmp/mimo_setup_stamps.bin")
os.environ["MPCQ_MIMO_SETUP_STAMPS"] = out
Ad, Bd = workload.quadrotor_plants(3, 0, B)
sh = workload.quadrotor_shared()
nx, ny = Ad.shape[1], np.asarray(sh["Cd"]).shape[0]
dev = torch.device("cuda:0")
tdev = lambda v: torch.as_tensor(np.ascontiguousarray(v, dtype=np.float64)).to(dev)  # noqa: E731
plant_d = [tdev(Ad), tdev(Bd)] + [
    torch.as_tensor(np.asarray(sh[k], dtype=np.float64)).to(dev).expand((B,) + np.asarray(sh[k]).shape).contiguous()
    for k in ("Cd", "Q", "R", "RD", "K", "K0", "w0")]
s = sm.BatchSolver(N * nu, 2 * N * nu, B, B, "f64", 0)
st = torch.cuda.current_stream(dev).cuda_stream
for _ in range(2):
    s.mimo_setup_plants_device(nx, nu, ny, N, *[t.data_ptr() for t in plant_d], stream=st)
torch.cuda.synchronize()
h = np.fromfile(out, dtype=np.int64).reshape(-1, 16)
names = {1: "plant data", 2: "transformations", 3: "Fx + QCS", 4: "setH + Fu + Frs", 5: "symmetrise",
         6: "Ruiz", 7: "outputs"}
tot = h[:, 7] - h[:, 0]
print(f"plants {len(h)}  setup cycles per plant: median {np.median(tot):.0f}  p90 {np.percentile(tot, 90):.0f}")
for k in range(1, 8):
    d = h[:, k] - h[:, k - 1]
    print(f"  {names[k]:18s} median {np.median(d):8.0f}  share {np.median(d) / np.median(tot):.3f}")
for k, nm in ((9, "pass-1 first barrier"), (10, "pass-1 A norms + cost"), (11, "pass-1 D, E update")):
    d = h[:, k] - h[:, k - 1]
    print(f"  {nm:22s} median {np.median(d):8.0f}")

# co-residency: workgroups of one CU (HW_ID cu/sh/se fields + XCC) overlapping in s_memrealtime (100 MHz)
hw, xcc, t0, t1 = h[:, 12], h[:, 13], h[:, 14], h[:, 15]
cu = (xcc & 0xF) * 4096 + ((hw >> 8) & 0xF) + 16 * ((hw >> 12) & 0x1) + 32 * ((hw >> 13) & 0x7)
ev = np.concatenate([np.stack([t0, np.ones_like(t0), cu], 1), np.stack([t1, -np.ones_like(t1), cu], 1)])
ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
from collections import defaultdict
live, peak = defaultdict(int), defaultdict(int)
for tt, d, c in ev:
    live[c] += d
    peak[c] = max(peak[c], live[c])
pk = np.array(list(peak.values()))
print(f"CUs seen {len(pk)}; workgroups resident at once per CU: max {pk.max()} median {np.median(pk):.0f}")
print(f"kernel span {(t1.max() - t0.min()) / 100:.0f} us; mean workgroup {(t1 - t0).mean() / 100:.1f} us")
