#!/bin/bash
# Round-4 pass x (dev tool): HEAD's GPU suite + smoke, the driver's default bench, and the stream line
# with its new default plants per wave.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/ -v -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/x_default.json 2> gpurun_out/x_default.err || exit $?
timeout -k 10 300 python bench.py --workload stream --steps 3 --warmup 1 > gpurun_out/x_stream.json 2> gpurun_out/x_stream.err || exit $?
for rep in 1 2 3; do
  timeout -k 10 200 python bench.py --workload perplant --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/x_pp_$rep.json 2>> gpurun_out/x_pp.err || exit $?
done
exit 0
