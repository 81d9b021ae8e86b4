#!/bin/bash
# Round-4 pass u (dev tool): the f64 check iteration reusing the stacked loop's carried -g + S x': GPU
# suite, then A/B against libmpcq_b.so (before) in mixed and f64.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/ -v -s -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do
  for v in b:solvempc_amd/libmpcq_b.so sx:solvempc_amd/libmpcq.so; do
    name=${v%%:*}; lib=${v#*:}
    for dt in mixed f64; do
      MPCQ_LIBRARY=$lib timeout -k 10 120 python bench.py --dtype $dt --steps 20 --warmup 3 --cpu-seconds 0 --variants 0 > gpurun_out/u_${name}_${dt}_$rep.json 2>> gpurun_out/u.err || exit $?
    done
  done
done
exit 0
