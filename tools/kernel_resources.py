"""Static resource table of the built device code (dev tool, CPU only): for every kernel in the gfx950 code
objects of solvempc_amd/csrc/build/*.hip.o, its scratch bytes per lane (.private_segment_fixed_size), VGPR /
AGPR counts, spilled VGPRs and LDS bytes, read from the AMDGPU metadata note.  The numbers match rocprofv3's
Scratch_Size / VGPR columns of the kernel traces under profiles/ without a GPU run.

usage: python tools/kernel_resources.py [--filter SUBSTR] [--json]"""
import argparse
import json
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
BUILD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "solvempc_amd", "csrc", "build")
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
FIELDS = {"scratch": r"\.private_segment_fixed_size:\s+(\d+)", "vgpr": r"\.vgpr_count:\s+(\d+)",
          "agpr": r"\.agpr_count:\s+(\d+)", "vgpr_spill": r"\.vgpr_spill_count:\s+(\d+)",
          "sgpr_spill": r"\.sgpr_spill_count:\s+(\d+)", "lds": r"\.group_segment_fixed_size:\s+(\d+)"}


def demangle(names):
    out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True)
    return out.stdout.splitlines() if out.returncode == 0 else names


def kernels(obj):
    """[(mangled name, {field: int})] of one object file's gfx950 code object."""
    with tempfile.TemporaryDirectory() as d:
        fat, co = os.path.join(d, "fat"), os.path.join(d, "co")
        if subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj, os.path.join(d, "o")],
                          capture_output=True).returncode:
            return []
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                        f"--targets={TARGET}", f"--output={co}"], check=True, capture_output=True)
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True,
                               text=True).stdout
    res = []
    for blk in notes.split("  - ."):
        m = re.search(r"\.name:\s+(\S+)", blk)
        if not m or not re.search(FIELDS["scratch"], blk):
            continue
        vals = {}
        for k, pat in FIELDS.items():
            f = re.search(pat, blk)
            vals[k] = int(f.group(1)) if f else 0
        res.append((m.group(1), vals))
    return res


def table(filt=""):
    rows = []
    for f in sorted(os.listdir(BUILD)):
        if f.endswith(".hip.o"):
            for name, vals in kernels(os.path.join(BUILD, f)):
                rows.append({"object": f[:-6], "mangled": name, **vals})
    for r, d in zip(rows, demangle([r["mangled"] for r in rows])):
        r["kernel"] = d
    return [r for r in rows if filt in r["kernel"]]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--filter", default="")
    ap.add_argument("--json", action="store_true")
    args = ap.parse_args()
    rows = table(args.filter)
    if args.json:
        json.dump(rows, sys.stdout, indent=1)
        return
    print(f"{'scratch':>7} {'vgpr':>4} {'agpr':>4} {'spill':>5} {'lds':>6}  kernel")
    for r in rows:
        print(f"{r['scratch']:7d} {r['vgpr']:4d} {r['agpr']:4d} {r['vgpr_spill']:5d} {r['lds']:6d}  {r['kernel']}")


if __name__ == "__main__":
    main()
