set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r05ah
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "plant" > gpurun_out/r05ah/tests.log 2>&1 || { tail -30 gpurun_out/r05ah/tests.log; exit 1; }
for rep in 1 2 3; do
  for v in old new; do
    if [ $v = old ]; then L=$GRAFT_REPO_ROOT/tools/ab_base/libmpcq.so; else L=$GRAFT_REPO_ROOT/solvempc_amd/libmpcq.so; fi
    MPCQ_LIBRARY=$L timeout -k 10 200 python bench.py --workload perplant --steps 10 --warmup 2 --cpu-seconds 0 --variants 0 > gpurun_out/r05ah/pp_${v}_$rep.json 2>> gpurun_out/r05ah/ab.err || exit 1
  done
done
