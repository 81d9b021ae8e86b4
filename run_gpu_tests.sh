#!/bin/bash
# GPU driver: tests, smoke, a short bench per dtype.  Each GPU step has its own time limit and the
# script stops at the first abnormal exit (fault/abort/timeout); plain test failures (rc 1) go on.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu.py -q -m gpu -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" >> gpurun_out/smoke.log
if [ $rc -gt 1 ]; then exit $rc; fi
for dt in f64 f32; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 1 --dtype $dt --cpu-seconds 3 > gpurun_out/bench_$dt.json 2> gpurun_out/bench_$dt.err
  rc=$?; if [ $rc -ne 0 ]; then echo "bench $dt rc=$rc" >> gpurun_out/bench_$dt.err; exit $rc; fi
done
exit 0
