#!/bin/bash
# Round-4 pass zk (dev tool): tile kernel with the check settings in LDS: the GPU suite, then
# interleaved config-2 lines (mixed, f64, f32), base library vs new.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/ -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/zk_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/zk_tests.log
[ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for v in base new; do
    lib=solvempc_amd/libmpcq.so; [ $v = base ] && lib=solvempc_amd/libmpcq_base.so
    for dt in mixed f64 f32; do
      MPCQ_LIBRARY=$lib timeout -k 10 120 python bench.py --dtype $dt --steps 20 --warmup 2 --cpu-seconds 0 --variants 0 > gpurun_out/zk_${dt}_${v}_$rep.json 2>> gpurun_out/zk.err || exit $?
    done
  done
done
exit 0
