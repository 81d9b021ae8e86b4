#!/bin/bash
# Debug build of libmpcq.so with one extra define on mpcq_mimo.hip (dev tool; needs the regular build's
# objects).  usage: bash tools/build_dbg.sh MPCQ_GJ_STAMPS  ->  tools/dbg/libmpcq.so (MPCQ_LIBRARY=...)
set -e
cd "$(dirname "$0")/../solvempc_amd/csrc"
mkdir -p ../../tools/dbg
/opt/rocm/bin/hipcc -O3 -ffp-contract=off -fno-slp-vectorize -std=c++17 -fPIC --offload-arch=gfx950 $(for d in "$@"; do printf -- "-D%s " "$d"; done) -c mpcq_mimo.hip -o ../../tools/dbg/mpcq_mimo.o
objs=$(ls build/*.o | grep -v mpcq_mimo)
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../../tools/dbg/libmpcq.so $objs ../../tools/dbg/mpcq_mimo.o
