#!/bin/bash
# Round-4 pass n (dev tool): GPU suite on HEAD's library, A/B of the prologue prefetch (libmpcq_stk.so =
# the library before it, at the same MPCQ_MIX_R), the driver's default bench line and its kernel trace.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/ -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
for rep in 1 2 3; do
  while read -r name lib dt envs; do
    [ -z "$name" ] && continue
    env MPCQ_LIBRARY=$lib $envs timeout -k 10 120 python bench.py --dtype $dt --steps 20 --warmup 3 --cpu-seconds 0 --variants 0 > gpurun_out/ab_${name}_$rep.json 2>> gpurun_out/ab.err || exit $?
  done <<AB
stk_mixed solvempc_amd/libmpcq_stk.so mixed MPCQ_MIX_R=5
pf_mixed solvempc_amd/libmpcq.so mixed
stk_f64 solvempc_amd/libmpcq_stk.so f64
pf_f64 solvempc_amd/libmpcq.so f64
stk_f32 solvempc_amd/libmpcq_stk.so f32
pf_f32 solvempc_amd/libmpcq.so f32
AB
done
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit $?
timeout -k 10 300 python bench.py --workload perplant --steps 5 --warmup 2 > gpurun_out/bench_perplant.json 2> gpurun_out/bench_perplant.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 5 --warmup 1 --cpu-seconds 0 > gpurun_out/prof.log 2>&1 || exit $?
exit 0
