#!/bin/bash
# GPU driver: tests, smoke, a short bench per dtype, then a rocprofv3 kernel trace of the bench.
# Each GPU step has its own time limit and the script stops at the first abnormal exit
# (test failure, fault, abort, timeout).
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/ -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" >> gpurun_out/smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
for dt in ${BENCH_DTYPES:-f32 f64}; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 1 --dtype $dt --cpu-seconds ${CPU_SECONDS:-3} > gpurun_out/bench_$dt.json 2> gpurun_out/bench_$dt.err
  rc=$?; if [ $rc -ne 0 ]; then echo "bench $dt rc=$rc" >> gpurun_out/bench_$dt.err; exit $rc; fi
done
if [ -n "$PROFILE" ]; then
  for dt in ${BENCH_DTYPES:-f32 f64}; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$dt -o run -- python bench.py --steps 5 --warmup 1 --dtype $dt --cpu-seconds 0 > gpurun_out/prof_$dt.log 2>&1
    rc=$?; if [ $rc -ne 0 ]; then echo "rocprof $dt rc=$rc" >> gpurun_out/prof_$dt.log; exit $rc; fi
  done
fi
exit 0
