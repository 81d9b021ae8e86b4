#!/bin/bash
# Instruction-fetch stall and I-cache counters of the cfg2 bench, one rocprofv3 pass per counter set.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/pmc_ic
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_IFETCH --output-format csv -d gpurun_out/pmc_ic/a -o run -- python bench.py --steps 2 --warmup 1 --cpu-seconds 0 > gpurun_out/pmc_ic/a.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ --output-format csv -d gpurun_out/pmc_ic/b -o run -- python bench.py --steps 2 --warmup 1 --cpu-seconds 0 > gpurun_out/pmc_ic/b.log 2>&1 || exit $?
