#!/bin/bash
# Phase-schedule A/B (kernel traces) + prologue sub-part stamps (tools/dbg/r*) in one call (dev tool).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
PFX=r PARTS="10 11 12 13 14" bash tools/gpu_info_parts.sh || exit $?
bash tools/gpu_ab_run.sh
