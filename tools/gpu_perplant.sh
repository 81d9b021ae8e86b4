#!/bin/bash
# GPU: per-plant (config 3) tests, full GPU suite, perplant bench per dtype, rocprof kernel stats.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/ -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for dt in ${BENCH_DTYPES:-f32 f64}; do
  timeout -k 10 300 python bench.py --workload perplant --steps 3 --warmup 1 --dtype $dt --cpu-seconds ${CPU_SECONDS:-3} > gpurun_out/bench_pp_$dt.json 2> gpurun_out/bench_pp_$dt.err
  rc=$?; if [ $rc -ne 0 ]; then echo "bench rc=$rc" >> gpurun_out/bench_pp_$dt.err; exit $rc; fi
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_pp -o run -- python bench.py --workload perplant --steps 3 --warmup 1 --dtype f32 --cpu-seconds 0 > gpurun_out/prof_pp.log 2>&1
