#!/bin/bash
# Round-4 pass y (dev tool): rocprofv3 kernel stats + trace of the config-4 and config-5 bench lines.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_y5 -o run -- python bench.py --workload stream --steps 2 --warmup 1 --cpu-seconds 0 > gpurun_out/prof_y5.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_y4 -o run -- python bench.py --workload quadrotor --steps 2 --warmup 1 --cpu-seconds 0 > gpurun_out/prof_y4.log 2>&1 || exit $?
exit 0
