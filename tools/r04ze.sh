#!/bin/bash
# Round-4 pass ze (dev tool): DPP moves without an "old" operand (full permutations; bound_ctrl zero
# fill for the MIMO row shifts): the whole GPU suite, then interleaved lines, base library vs new.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/ -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/ze_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/ze_tests.log
[ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for v in base new; do
    lib=solvempc_amd/libmpcq.so; [ $v = base ] && lib=solvempc_amd/libmpcq_base.so
    MPCQ_LIBRARY=$lib timeout -k 10 200 python bench.py --workload quadrotor --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/ze_q_${v}_$rep.json 2>> gpurun_out/ze.err || exit $?
    MPCQ_LIBRARY=$lib timeout -k 10 200 python bench.py --workload perplant --steps 5 --warmup 2 --cpu-seconds 0 --variants 0 > gpurun_out/ze_p_${v}_$rep.json 2>> gpurun_out/ze.err || exit $?
    MPCQ_LIBRARY=$lib timeout -k 10 200 python bench.py --workload perplant --dtype f32 --steps 5 --warmup 2 --cpu-seconds 0 --variants 0 > gpurun_out/ze_p32_${v}_$rep.json 2>> gpurun_out/ze.err || exit $?
  done
done
exit 0
