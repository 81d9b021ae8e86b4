#!/bin/bash
# The driver's round-end bench invocation (default workload) and its rocprofv3 kernel stats.
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out/dl
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/dl/bench.json 2> gpurun_out/dl/bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dl/prof -o run -- python bench.py --steps 5 --warmup 1 --cpu-seconds 0 > gpurun_out/dl/prof.log 2>&1
