#!/bin/bash
# Round-4 pass t (dev tool): the tile kernel with W, W' and the front-end rows out of LDS (a workgroup within
# a third of the CU's LDS): GPU suite, then A/B against libmpcq_s.so (before) in mixed, f64 and f32.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/ -v -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do
  for v in s:solvempc_amd/libmpcq_s.so lds:solvempc_amd/libmpcq.so; do
    name=${v%%:*}; lib=${v#*:}
    for dt in mixed f64 f32; do
      MPCQ_LIBRARY=$lib timeout -k 10 120 python bench.py --dtype $dt --steps 20 --warmup 3 --cpu-seconds 0 --variants 0 > gpurun_out/t_${name}_${dt}_$rep.json 2>> gpurun_out/t.err || exit $?
    done
  done
done
exit 0
