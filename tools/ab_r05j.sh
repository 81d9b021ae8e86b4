#!/bin/bash
# old/new library A/B over the cfg2 (mixed, f64) and cfg5 benches, interleaved
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r05j
for rep in 1 2 3; do
  for lib in old new; do
    L=tools/ab_old/libmpcq.so; [ $lib = new ] && L=solvempc_amd/libmpcq.so
    MPCQ_LIBRARY=$L timeout -k 10 120 python bench.py --dtype mixed --steps 20 --warmup 3 --cpu-seconds 0 --variants 0 > gpurun_out/r05j/ab_${lib}_mixed_$rep.json 2>> gpurun_out/r05j/ab.err || exit 1
    MPCQ_LIBRARY=$L timeout -k 10 120 python bench.py --dtype f64 --steps 20 --warmup 3 --cpu-seconds 0 --variants 0 > gpurun_out/r05j/ab_${lib}_f64_$rep.json 2>> gpurun_out/r05j/ab.err || exit 1
    if [ $rep -le 2 ]; then
      MPCQ_LIBRARY=$L timeout -k 10 120 python bench.py --workload stream --cpu-seconds 0 --variants 0 > gpurun_out/r05j/ab_${lib}_stream_$rep.json 2>> gpurun_out/r05j/ab.err || exit 1
    fi
  done
done
