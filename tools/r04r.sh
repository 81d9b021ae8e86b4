#!/bin/bash
# Round-4 pass r (dev tool): GPU suite + smoke on HEAD's library, A/B of the per-plant kernel's DPP / loop
# changes (libmpcq_pp0.so = before), and its stage isolation.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/ -v -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
for rep in 1 2 3; do
  for v in pp0:solvempc_amd/libmpcq_pp0.so new:solvempc_amd/libmpcq.so; do
    name=${v%%:*}; lib=${v#*:}
    MPCQ_LIBRARY=$lib timeout -k 10 200 python bench.py --workload perplant --dtype f64 --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/pp_${name}_$rep.json 2>> gpurun_out/pp.err || exit $?
  done
done
timeout -k 10 300 python tools/plant_profile.py > gpurun_out/plant_profile.txt 2>&1 || exit $?
exit 0
