#!/bin/bash
# Round-4 workload sweep (dev tool): config 3 strong-scaled at N = 1 (all 1,048,576 plants on one GPU),
# config 3 weak (131,072), config 4, config 5, each one bench line.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --workload perplant --scaling strong --steps 3 --warmup 1 --cpu-seconds 4 > gpurun_out/k_cfg3_strong.json 2> gpurun_out/k_cfg3_strong.err || exit $?
timeout -k 10 300 python bench.py --workload perplant --steps 10 --warmup 2 --cpu-seconds 4 > gpurun_out/k_cfg3.json 2> gpurun_out/k_cfg3.err || exit $?
timeout -k 10 300 python bench.py --workload quadrotor --steps 3 --warmup 1 --cpu-seconds 4 > gpurun_out/k_cfg4.json 2> gpurun_out/k_cfg4.err || exit $?
timeout -k 10 300 python bench.py --workload stream --steps 3 --warmup 1 --cpu-seconds 4 > gpurun_out/k_cfg5.json 2> gpurun_out/k_cfg5.err || exit $?
exit 0
