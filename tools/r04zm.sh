#!/bin/bash
# Round-4 pass zm (dev tool): per-plant kernel with its check settings in LDS: the per-plant GPU tests on
# the new library, then interleaved config-3 lines (f64 default, f32), HEAD library vs new.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
NEW=solvempc_amd/libmpcq_plantlds.so
MPCQ_LIBRARY=$NEW timeout -k 10 300 python -u -m pytest tests/test_plants_step.py tests/test_gpu.py -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread -k "plant or config3" > gpurun_out/zm_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/zm_tests.log
[ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for v in base new; do
    lib=solvempc_amd/libmpcq.so; [ $v = new ] && lib=$NEW
    MPCQ_LIBRARY=$lib timeout -k 10 200 python bench.py --workload perplant --steps 5 --warmup 2 --cpu-seconds 0 --variants 0 > gpurun_out/zm_p_${v}_$rep.json 2>> gpurun_out/zm.err || exit $?
    MPCQ_LIBRARY=$lib timeout -k 10 200 python bench.py --workload perplant --dtype f32 --steps 5 --warmup 2 --cpu-seconds 0 --variants 0 > gpurun_out/zm_p32_${v}_$rep.json 2>> gpurun_out/zm.err || exit $?
  done
done
exit 0
