#!/bin/bash
# One cfg2 solve with per-wave phase stamps (MPCQ_TILE_STAMPS) and their summary (tools/stamps.py).
# usage: bash tools/gpu_stamps.sh <tag> [bench args]
cd "$GRAFT_REPO_ROOT" || exit 2
t=${1:-st}; shift
o=gpurun_out/$t; mkdir -p "$o"
MPCQ_TILE_STAMPS=$o/stamps.bin timeout -k 10 120 python bench.py --steps 1 --warmup 1 --cpu-seconds 0 "$@" > $o/bench.json 2> $o/bench.err || exit $?
python tools/stamps.py $o/stamps.bin > $o/stamps.txt
