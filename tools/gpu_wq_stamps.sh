#!/bin/bash
# One cfg2 solve with work-queue stamps (MPCQ_TILE_STAMPS) and its summary.  usage: bash tools/gpu_wq_stamps.sh <tag>
cd "$GRAFT_REPO_ROOT" || exit 2
o=gpurun_out/${1:-wqs}; mkdir -p "$o"
MPCQ_TILE_STAMPS=$o/stamps.bin timeout -k 10 120 python bench.py --steps 1 --warmup 1 --cpu-seconds 0 > $o/bench.json 2> $o/bench.err || exit $?
python tools/wq_stamps.py $o/stamps.bin > $o/stamps.txt
