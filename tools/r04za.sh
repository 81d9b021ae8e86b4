#!/bin/bash
# Round-4 pass za (dev tool): the one-barrier MIMO iteration (rows permuted by component for n_u = 4
# with a diagonal K0): MIMO GPU tests, then interleaved config-4 lines, base library vs new.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_mimo.py -v -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/${TAG:-za}_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/${TAG:-za}_tests.log
[ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for v in base new; do
    lib=solvempc_amd/libmpcq.so; [ $v = base ] && lib=solvempc_amd/libmpcq_base.so
    MPCQ_LIBRARY=$lib timeout -k 10 200 python bench.py --workload quadrotor --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/${TAG:-za}_${v}_$rep.json 2>> gpurun_out/${TAG:-za}.err || exit $?
  done
done
exit 0
