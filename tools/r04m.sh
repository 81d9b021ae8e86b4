#!/bin/bash
# Round-4 pass m (dev tool): per-wave stamps of the mixed tile kernel's info iterations, whole
# (tools/dbglib_i0) and split into parts 1-5 (MPCQ_INFO_PART, tools/dbglib_iP).
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
export MPCQ_MIX_R=5
for p in 0 1 2 3 4 5; do
  DTYPES=mixed LIB=tools/dbglib_i$p/libmpcq.so TAG=_i$p bash tools/stamps_run.sh || exit $?
done
exit 0
