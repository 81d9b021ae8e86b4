#!/bin/bash
# Debug build of libmpcq.so (dev tool; needs the regular build's objects): mpcq_api.cpp and one kernel
# source (default mpcq_tile_f32.hip; SRC=... to pick another) recompiled with -DMPCQ_DEBUG_HOOKS (the
# stamp / profiling dumps, mpcq_api.cpp "Test hooks") plus the extra defines given.
# usage: [SRC=mpcq_mimo.hip] bash tools/build_dbg.sh [MPCQ_INFO_STAMPS ...]  ->  tools/dbglib/libmpcq.so
#        then MPCQ_LIBRARY=tools/dbglib/libmpcq.so MPCQ_TILE_STAMPS=out.bin python ...
set -e
cd "$(dirname "$0")/../solvempc_amd/csrc"
D=../../${DBGDIR:-tools/dbglib}; mkdir -p $D
SRC=${SRC:-mpcq_tile_f32.hip}
DEFS="-DMPCQ_DEBUG_HOOKS $(for d in "$@"; do printf -- "-D%s " "$d"; done)"
FL="-O3 -ffp-contract=off -fno-slp-vectorize -std=c++17 -fPIC --offload-arch=gfx950"
/opt/rocm/bin/hipcc $FL $DEFS -c $SRC -o $D/dbg_src.o
/opt/rocm/bin/hipcc $FL $DEFS -c mpcq_api.cpp -o $D/dbg_api.o
objs=$(ls build/*.o | grep -v -e "$SRC" -e mpcq_api.cpp)
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $D/libmpcq.so $objs $D/dbg_src.o $D/dbg_api.o
