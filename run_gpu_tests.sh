#!/bin/bash
# GPU driver: tests, smoke, a short bench per dtype, then (PROFILE=1) a rocprofv3 kernel trace of the
# bench.  Each GPU step has its own time limit and the script stops at the first abnormal exit
# (test failure, fault, abort, timeout).
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/ -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" >> gpurun_out/smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
for wl in ${BENCH_WORKLOADS:-cfg2}; do
  [ "$wl" = none ] && continue
  timeout -k 10 300 python bench.py --workload $wl --steps ${BENCH_STEPS:-10} --warmup 2 --cpu-seconds ${CPU_SECONDS:-4} > gpurun_out/bench_$wl.json 2> gpurun_out/bench_$wl.err
  rc=$?; if [ $rc -ne 0 ]; then echo "bench $wl rc=$rc" >> gpurun_out/bench_$wl.err; exit $rc; fi
done
if [ -n "$PROFILE" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 5 --warmup 1 --cpu-seconds 0 > gpurun_out/prof.log 2>&1
  rc=$?; if [ $rc -ne 0 ]; then echo "rocprof rc=$rc" >> gpurun_out/prof.log; exit $rc; fi
fi
exit 0
