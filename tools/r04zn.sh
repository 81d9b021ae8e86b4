#!/bin/bash
# Round-4 pass zn (dev tool): pass zm (per-plant settings in LDS, A/B), then the rocprofv3 kernel stats
# of the config-4 bench line.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/r04zm.sh || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_zl -o run -- python bench.py --workload quadrotor --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/zl_q_prof.json 2> gpurun_out/zl.err || exit $?
exit 0
