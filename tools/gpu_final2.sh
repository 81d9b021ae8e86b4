#!/bin/bash
# Round-end evidence: gpu_round.sh (tests, smoke, every bench, kernel stats) + per-plant setup stage cycles.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
bash tools/gpu_round.sh ${1:-final} || exit $?
timeout -k 10 120 python tools/setup_prof.py 4096 > gpurun_out/${1:-final}/setup_stage_cycles.txt 2>&1
