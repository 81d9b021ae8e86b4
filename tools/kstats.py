"""Register, scratch and LDS use of every kernel of one HIP source (dev tool): compiles it for gfx950 with
-save-temps into a scratch directory and reads the code object metadata of the .s file.
usage: python tools/kstats.py solvempc_amd/csrc/mpcq_plant.hip [name_substring] [-Dextra ...]"""
import glob
import os
import re
import subprocess
import sys
import tempfile

src = os.path.abspath(sys.argv[1])
pat = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("-") else ""
extra = [a for a in sys.argv[2:] if a.startswith("-")]
d = tempfile.mkdtemp(prefix="kstats_")
flags = ["-O3", "-ffp-contract=off", "-fno-slp-vectorize", "-std=c++17", "-fPIC", "--offload-arch=gfx950",
         "--cuda-device-only", "-save-temps", "-c", "-o", os.path.join(d, "k.o")]
subprocess.run(["/opt/rocm/bin/hipcc", *flags, *extra, src], cwd=d, check=True)
s = open(glob.glob(os.path.join(d, "*gfx950*.s"))[0]).read()
meta = s[s.index("amdhsa.kernels:"):]
for blk in re.split(r"\n  - ", meta)[1:]:
    g = lambda k: (re.search(r"\." + k + r":\s+(\S+)", blk) or [None, "?"])[1]  # noqa: E731
    name = g("name")
    if pat and pat not in name:
        continue
    dem = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
    print(f"vgpr {g('vgpr_count'):>4} agpr {g('agpr_count'):>4} sgpr {g('sgpr_count'):>4} "
          f"scratch {g('private_segment_fixed_size'):>5} lds {g('group_segment_fixed_size'):>6}  {dem[:150]}")
