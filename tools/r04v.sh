#!/bin/bash
# Round-4 pass v (dev tool): plants per wave of the tile stream mode (MPCQ_STREAM_CPW) for the fp64 and
# mixed streams (config 5; the default is ceil(batch / SIMDs) = 4).
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  for cpw in 2 4 8; do
    for dt in f64 mixed; do
      MPCQ_STREAM_CPW=$cpw timeout -k 10 200 python bench.py --workload stream --dtype $dt --steps 2 --warmup 1 --cpu-seconds 0 > gpurun_out/v_${dt}_cpw${cpw}_$rep.json 2>> gpurun_out/v.err || exit $?
    done
  done
done
exit 0
