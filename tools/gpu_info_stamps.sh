#!/bin/bash
# Tile-kernel stamps with the info-iteration cycle counter (MPCQ_INFO_STAMPS debug build in tools/dbg).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
MPCQ_LIBRARY=$PWD/tools/dbg/libmpcq.so bash tools/gpu_stamps.sh ${1:-sti}
