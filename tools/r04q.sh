#!/bin/bash
# Round-4 pass q (dev tool): the mixed tile stream mode (config 5): stream GPU tests, then bench lines of
# the stream in mixed (with its oracle parity block), f64 and f32.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/ -v -s -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread -k stream > gpurun_out/stream_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/stream_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --workload stream --dtype mixed --steps 3 --warmup 1 --cpu-seconds 4 > gpurun_out/st_mixed.json 2> gpurun_out/st.err || exit $?
for rep in 1 2; do
  for dt in mixed f64 f32; do
    timeout -k 10 300 python bench.py --workload stream --dtype $dt --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/st_${dt}_$rep.json 2>> gpurun_out/st.err || exit $?
  done
done
exit 0
