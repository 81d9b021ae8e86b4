#!/bin/bash
# A/B library (dev tool): libmpcq.so with the given kernel sources taken from git revision REV (the rest from
# the current build's objects) -> tools/ab_NAME/libmpcq.so.  usage: tools/ablib.sh NAME REV src.hip [...]
set -e
name=$1; rev=$2; shift 2
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
git -C "$root" archive "$rev" solvempc_amd/csrc include | tar -x -C "$tmp"
cd "$root/solvempc_amd/csrc"
FL="-O3 -ffp-contract=off -fno-slp-vectorize -std=c++17 -fPIC --offload-arch=gfx950"
objs=$(ls build/*.o)
for src in "$@"; do
  /opt/rocm/bin/hipcc $FL -c "$tmp/solvempc_amd/csrc/$src" -o "$tmp/$src.o"
  objs=$(echo "$objs" | grep -v "build/$src.o")
  objs="$objs $tmp/$src.o"
done
mkdir -p "$root/tools/ab_$name"
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "$root/tools/ab_$name/libmpcq.so" $objs
rm -rf "$tmp"
