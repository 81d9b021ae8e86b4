#!/bin/bash
# GPU: config-4 (quad-rotor MIMO) tests, the quadrotor bench, rocprof kernel stats.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_mimo.py -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/quad_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/quad_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --workload quadrotor --steps ${STEPS:-3} --warmup 1 --cpu-seconds ${CPU_SECONDS:-5} > gpurun_out/bench_quad.json 2> gpurun_out/bench_quad.err
rc=$?; if [ $rc -ne 0 ]; then echo "bench rc=$rc" >> gpurun_out/bench_quad.err; exit $rc; fi
if [ -n "$NOPROF" ]; then exit 0; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_quad -o run -- python bench.py --workload quadrotor --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/prof_quad.log 2>&1
