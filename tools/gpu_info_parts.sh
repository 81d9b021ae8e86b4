#!/bin/bash
# Info-iteration cost by part (MPCQ_INFO_PART debug builds in tools/dbg/p*): tile stamps per part.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
for p in ${PARTS:-1 2 3 5}; do
  MPCQ_LIBRARY=$PWD/tools/dbg/${PFX:-p}$p/libmpcq.so bash tools/gpu_stamps.sh ${PFX:-p}art$p || exit $?
done
