#!/bin/bash
# Debug build of libmpcq.so with extra defines on one source (default mpcq_mimo.hip; SRC=... to pick
# another) (dev tool; needs the regular build's objects).
# usage: [SRC=mpcq_tile_f32.hip] bash tools/build_dbg.sh MPCQ_GJ_STAMPS  ->  tools/dbg/libmpcq.so (MPCQ_LIBRARY=...)
set -e
cd "$(dirname "$0")/../solvempc_amd/csrc"
mkdir -p ../../tools/dbg
/opt/rocm/bin/hipcc -O3 -ffp-contract=off -fno-slp-vectorize -std=c++17 -fPIC --offload-arch=gfx950 $(for d in "$@"; do printf -- "-D%s " "$d"; done) -c ${SRC:-mpcq_mimo.hip} -o ../../tools/dbg/dbg_src.o
objs=$(ls build/*.o | grep -v "${SRC:-mpcq_mimo.hip}")
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../../tools/dbg/libmpcq.so $objs ../../tools/dbg/dbg_src.o
