#!/bin/bash
# gpu_check2.sh + the per-plant setup stage cycles (dev tool).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
bash tools/gpu_check2.sh || exit $?
timeout -k 10 120 python tools/setup_prof.py 4096 > gpurun_out/c2/setup_stage_cycles.txt 2>&1
